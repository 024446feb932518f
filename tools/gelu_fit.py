#!/usr/bin/env python3
"""Fit of the transcendental-free erf-GELU used by the GEMM epilogue (common.h gelu_poly16).

    xc = clamp(x, -A, A),  w = xc*xc - A^2/2           (one packed FMA)
    gelu(x) ~= x * (0.5 + xc * Q(w))                   (Horner in w, then one FMA and one MUL)

Q(w) ~= 0.5 * erf(xc / sqrt2) / xc, fitted in t = w / (A^2/2) in [-1, 1] (least squares on
Chebyshev nodes, weighted by u = xc^2 so the error of xc*Q is minimised), then rescaled to
monomials in w: the centred variable keeps the Horner sum as well conditioned as the Chebyshev
interval while needing no extra op to form it.
Prints the fp32 coefficients and the fp32-evaluated GELU error: max |err| and the fraction of
inputs whose bf16-rounded output differs from the bf16-rounded exact GELU.
"""
import argparse

import numpy as np
from scipy.special import erf


def fit(a: float, deg: int) -> np.ndarray:
    """Coefficients q_k (fp32) of Q(w) = sum q_k w^k, clamp A = a*sqrt2 in x-space."""
    A2 = 2 * a * a
    h = A2 / 2
    t = np.cos(np.linspace(0, np.pi, 8000))
    u = (t + 1) * h  # xc^2 in [0, A^2]
    x = np.sqrt(u)
    f = np.where(x > 0, 0.5 * erf(x / np.sqrt(2)) / np.maximum(x, 1e-30), 1 / np.sqrt(2 * np.pi))
    wgt = np.maximum(x, 1e-3)
    c, *_ = np.linalg.lstsq(np.polynomial.chebyshev.chebvander(t, deg) * wgt[:, None], f * wgt, rcond=None)
    mono_t = np.polynomial.chebyshev.cheb2poly(c)  # in t = w / h
    return (mono_t / h ** np.arange(deg + 1)).astype(np.float32)


def _fma32(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c).astype(np.float32)


def gelu_fp32(x: np.ndarray, a: float, q: np.ndarray) -> np.ndarray:
    """Bit-faithful emulation of gelu_poly16 (fp32 FMAs)."""
    x = x.astype(np.float32)
    A = np.float32(a * np.sqrt(2))
    h = np.float32(a * a)
    xc = np.clip(x, -A, A).astype(np.float32)
    w = _fma32(xc, xc, -np.float64(h))
    p = np.full_like(x, q[-1])
    for k in range(len(q) - 2, -1, -1):
        p = _fma32(p, w, np.float64(q[k]))
    f = _fma32(xc, p, 0.5)
    return (x * f).astype(np.float32)


def bf16(v: np.ndarray) -> np.ndarray:
    """Round fp32 -> bf16 (RNE), returned as fp32."""
    b = v.astype(np.float32).view(np.uint32).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000
    return b.astype(np.uint32).view(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", type=float, default=3.5, help="clamp of z = x/sqrt2")
    ap.add_argument("--deg", type=int, default=12)
    args = ap.parse_args()
    q = fit(args.a, args.deg)
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(2_000_000).astype(np.float32) * 2,
                        np.linspace(-12, 12, 800001).astype(np.float32)])
    ref = 0.5 * x.astype(np.float64) * (1 + erf(x.astype(np.float64) / np.sqrt(2)))
    g = gelu_fp32(x, args.a, q)
    err = np.abs(g - ref)
    mis = np.mean(bf16(g) != bf16(ref.astype(np.float32)))
    print("coefficients of Q(w):", ", ".join("%.9ef" % v for v in q))
    print("clamp %.9ef  A^2/2 %.9ef" % (np.float32(args.a * np.sqrt(2)), np.float32(args.a * args.a)))
    print(f"max |err| {err.max():.2e}; |x|<4: {err[np.abs(x) < 4].max():.2e}; "
          f"bf16 outputs differing from bf16(exact): {100 * mis:.3f} %")


if __name__ == "__main__":
    main()
