#!/usr/bin/env python3
"""LayerNorm-folding GEMMs vs their plain counterparts at the BERT-base bench shape.

Interleaved rounds in one process (guide §5.4 rule 24). For each encoder GEMM:
plain epilogue, LN-folding epilogue, and the folding kernel with its plain
epilogue (``gemm_ablate(7)``: staging + tile-loop structure only), plus the
LayerNorm and the statistics-finalize passes the folding trades.
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from agent_tpu_amd._native import native

    nat = native()
    assert nat.DEV_BUILD, "needs the dev extension: python -m agent_tpu_amd.csrc.build --dev (ablation schedules)"
    dev = torch.device("cuda", 0)
    M, H, I = a.rows * 128, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*shape, scale=1.0, dtype=torch.bfloat16):
        return (torch.randn(*shape, generator=g, device=dev) * scale).to(dtype)

    x768, x3072, res = r(M, H), r(M, I), r(M, H)
    wqkv, wo, w1, w2 = r(3 * H, H, scale=0.03), r(H, H, scale=0.03), r(I, H, scale=0.03), r(H, I, scale=0.03)
    bqkv, bo, b1, b2 = (r(n, scale=0.1, dtype=torch.float32) for n in (3 * H, H, I, H))
    gam, bet = 1 + r(H, scale=0.1, dtype=torch.float32), r(H, scale=0.1, dtype=torch.float32)
    cq, c1 = wqkv.float().sum(1), w1.float().sum(1)
    part = torch.empty((H // 256, M, 2), device=dev)
    fin = ops.ln_finalize(ops.ln_partials_ref(res.float()), H, 1e-12)
    cases = {
        "qkv": (lambda: ops.linear(x768, wqkv, bqkv),
                lambda: ops.linear_ln(x768, wqkv, bqkv, in_fin=fin, colsum=cq), 2 * M * H * 3 * H),
        "ffn1": (lambda: ops.linear(x768, w1, b1, act="gelu"),
                 lambda: ops.linear_ln(x768, w1, b1, act="gelu", in_fin=fin, colsum=c1), 2 * M * H * I),
        "o_stats": (lambda: ops.linear(x768, wo, bo, residual=res),
                    lambda: ops.linear_ln(x768, wo, bo, residual=res, part_out=part), 2 * M * H * H),
        "o_resnorm": (lambda: ops.linear(x768, wo, bo, residual=res),
                      lambda: ops.linear_ln(x768, wo, bo, residual=res, res_fin=fin, res_gamma=gam, part_out=part),
                      2 * M * H * H),
        "ffn2_resnorm": (lambda: ops.linear(x3072, w2, b2, residual=res),
                         lambda: ops.linear_ln(x3072, w2, b2, residual=res, res_fin=fin, res_gamma=gam, part_out=part),
                         2 * M * I * H),
    }
    times = {k: {"plain": [], "fold": [], "struct": [], "accinit": []} for k in cases}
    extra = {"layernorm": [], "finalize": []}
    for rd in range(a.rounds):
        for k in (list(cases) if rd % 2 == 0 else list(reversed(cases))):
            plain, fold, _ = cases[k]
            times[k]["plain"].append(timeit(plain, a.iters))
            times[k]["fold"].append(timeit(fold, a.iters))
            nat.gemm_ablate(7)
            times[k]["struct"].append(timeit(fold, a.iters))
            if k in ("qkv", "ffn1"):  # InNorm variant: accumulators started at -mu*colsum
                nat.gemm_ablate(8)
                times[k]["accinit"].append(timeit(fold, a.iters))
            nat.gemm_ablate(0)
        extra["layernorm"].append(timeit(lambda: ops.layernorm(x768, gam, bet, 1e-12), a.iters))
        extra["finalize"].append(timeit(lambda: ops.ln_finalize(part, H, 1e-12, out=fin), a.iters))
    out = {}
    for k, (_, _, fl) in cases.items():
        med = {v: statistics.median(t) for v, t in times[k].items() if t}
        out[k] = {f"{v}_us": round(t * 1000, 1) for v, t in med.items()}
        out[k].update({f"{v}_tflops": round(fl / t / 1e9, 1) for v, t in med.items()})
        print(k, json.dumps(out[k]), flush=True)
    for k, t in extra.items():
        out[k] = {"us": round(statistics.median(t) * 1000, 1)}
        print(k, json.dumps(out[k]), flush=True)
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
