#!/usr/bin/env python3
"""Fit of the transcendental-free erf-GELU used by the GEMM epilogue (common.h gelu_poly16).

erf(z) ~= z * P(t), z = clamp(x / sqrt(2), -a, a), t = 2 z^2 / a^2 - 1, P of degree `deg`
(least squares on Chebyshev nodes, weighted by z so the error of z*P is minimised).
Prints the fp32 monomial coefficients of P in t and the fp32-evaluated GELU error.
"""
import argparse

import numpy as np
from scipy.special import erf


def fit(a: float, deg: int) -> np.ndarray:
    z = np.cos(np.linspace(0, np.pi, 8000)) * a / 2 + a / 2
    t = 2 * z * z / (a * a) - 1
    f = np.where(z > 0, erf(z) / np.maximum(z, 1e-30), 2 / np.sqrt(np.pi))
    w = np.maximum(z, 1e-3)
    c, *_ = np.linalg.lstsq(np.polynomial.chebyshev.chebvander(t, deg) * w[:, None], f * w, rcond=None)
    return np.polynomial.chebyshev.cheb2poly(c).astype(np.float32)


def gelu_fp32(x: np.ndarray, a: float, m: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32)
    z = np.clip(x * np.float32(1 / np.sqrt(2)), -a, a).astype(np.float32)
    t = (z * z * np.float32(2 / (a * a)) - np.float32(1)).astype(np.float32)
    p = np.float32(m[-1])
    for k in range(len(m) - 2, -1, -1):
        p = (p * t + m[k]).astype(np.float32)
    hx = (np.float32(0.5) * x).astype(np.float32)
    return (hx * (z * p) + hx).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", type=float, default=3.5)
    ap.add_argument("--deg", type=int, default=12)
    args = ap.parse_args()
    m = fit(args.a, args.deg)
    x = np.linspace(-12, 12, 800001)
    ref = 0.5 * x * (1 + erf(x / np.sqrt(2)))
    err = np.abs(gelu_fp32(x, args.a, m) - ref)
    print("coefficients of P(t):", ", ".join("%.9ef" % v for v in m))
    # common.h evaluates in x-space: clamp x to +-a*sqrt2, t = x^2 / a^2 - 1, 1/sqrt2 folded into P
    mx = (m.astype(np.float64) * np.sqrt(0.5)).astype(np.float32)
    print("x-space (gelu_poly16):", ", ".join("%.9ef" % v for v in mx),
          "| clamp %.9ef  1/a^2 %.11ef" % (np.float32(args.a * np.sqrt(2)), np.float32(1 / args.a ** 2)))
    print(f"max |err| {err.max():.2e}; |x|<4: {err[np.abs(x) < 4].max():.2e}")


if __name__ == "__main__":
    main()
