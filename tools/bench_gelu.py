#!/usr/bin/env python3
"""A/B of the FFN1 GELU evaluation inside the LN-folded GEMM epilogue (BERT-base bench shape).

gemm_ablate: 0 = shipped (packed pairs, degree 10), 9 = scalar degree 10, 10 = packed degree 8,
11 = scalar degree 8 (common.h gelu_poly16_v). Interleaved rounds in one process; each variant
is also checked against an fp32 LayerNorm + linear + exact-erf GELU reference.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agent_tpu_amd import ops  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="0,9,10,11")
    a = ap.parse_args()
    from agent_tpu_amd._native import native

    nat = native()
    assert nat.DEV_BUILD, "needs the dev extension: python -m agent_tpu_amd.csrc.build --dev (ablation schedules)"
    dev = torch.device("cuda", 0)
    M, H, I = a.rows * 128, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*shape, scale=1.0, dtype=torch.bfloat16):
        return (torch.randn(*shape, generator=g, device=dev) * scale).to(dtype)

    x, w1 = r(M, H), r(I, H, scale=0.05)
    b1 = r(I, scale=0.1, dtype=torch.float32)
    c1 = w1.float().sum(1)
    fin = ops.ln_finalize(ops.ln_partials_ref(x.float()), H, 1e-12)
    variants = [int(v) for v in a.variants.split(",")]
    fold = lambda: ops.linear_ln(x, w1, b1, act="gelu", in_fin=fin, colsum=c1)  # noqa: E731
    # numerics on the first 4096 rows (fp32 reference of LN(x) . W^T + b -> exact GELU)
    xs = x[:4096].float()
    ln = (xs - xs.mean(1, keepdim=True)) / torch.sqrt(xs.var(1, unbiased=False, keepdim=True) + 1e-12)
    ref = torch.nn.functional.gelu(ln @ w1.float().t() + b1)
    errs = {}
    for v in variants:
        nat.gemm_ablate(v)
        out = fold()[:4096].float()
        errs[v] = float((out - ref).abs().max())
    nat.gemm_ablate(0)
    times = {v: [] for v in variants}
    for rd in range(a.rounds):
        for v in (variants if rd % 2 == 0 else list(reversed(variants))):
            nat.gemm_ablate(v)
            times[v].append(timeit(fold, a.iters))
    nat.gemm_ablate(0)
    fl = 2 * M * H * I
    out = {}
    for v, t in times.items():
        med = statistics.median(t)
        out[str(v)] = {"us": round(med * 1000, 1), "min_us": round(min(t) * 1000, 1),
                       "tflops": round(fl / med / 1e9, 1), "max_abs_err": errs[v]}
        print(v, json.dumps(out[str(v)]), flush=True)
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
