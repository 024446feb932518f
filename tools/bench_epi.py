#!/usr/bin/env python3
"""Where the LN-folding GEMMs' epilogue time goes (dev build, timing only).

For each encoder GEMM of the BERT-base bench shape (M = 131072), interleaved rounds in
one process: the full kernel, the kernel whose epilogue computes everything but issues
no global stores (``gemm_ablate(12)``), and the kernel with no epilogue at all
(``gemm_ablate(13)``, accumulators kept live). full - nostore = the exposed store cost,
nostore - noepi = the epilogue's math, LDS transposes and residual loads.
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
    assert nat.DEV_BUILD, "needs a dev extension (python -m agent_tpu_amd.csrc.build --dev)"
    dev = torch.device("cuda", 0)
    M, H, I = a.rows * 128, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*shape, scale=1.0, dtype=torch.bfloat16):
        return (torch.randn(*shape, generator=g, device=dev) * scale).to(dtype)

    x768, x3072, res = r(M, H), r(M, I), r(M, H)
    wqkv, wo, w1, w2 = r(3 * H, H, scale=0.03), r(H, H, scale=0.03), r(I, H, scale=0.03), r(H, I, scale=0.03)
    bqkv, bo, b1, b2 = (r(n, scale=0.1, dtype=torch.float32) for n in (3 * H, H, I, H))
    gam = 1 + r(H, scale=0.1, dtype=torch.float32)
    cq, c1 = wqkv.float().sum(1), w1.float().sum(1)
    part = torch.empty((H // 256, M, 2), device=dev)
    fin = ops.ln_finalize(ops.ln_partials_ref(res.float()), H, 1e-12)
    cases = {
        "qkv": (lambda: ops.linear_ln(x768, wqkv, bqkv, in_fin=fin, colsum=cq), 2 * M * H * 3 * H),
        "ffn1": (lambda: ops.linear_ln(x768, w1, b1, act="gelu", in_fin=fin, colsum=c1), 2 * M * H * I),
        "o_resnorm": (lambda: ops.linear_ln(x768, wo, bo, residual=res, res_fin=fin, res_gamma=gam, part_out=part),
                      2 * M * H * H),
        "ffn2_resnorm": (lambda: ops.linear_ln(x3072, w2, b2, residual=res, res_fin=fin, res_gamma=gam,
                                               part_out=part), 2 * M * I * H),
    }
    modes = {"full": 0, "nostore": 12, "noepi": 13}
    times = {k: {m: [] for m in modes} for k in cases}
    for rd in range(a.rounds):
        for k in (list(cases) if rd % 2 == 0 else list(reversed(cases))):
            for m, ab in modes.items():
                nat.gemm_ablate(ab)
                times[k][m].append(timeit(cases[k][0], a.iters))
            nat.gemm_ablate(0)
    out = {}
    for k, (_, fl) in cases.items():
        med = {m: statistics.median(t) for m, t in times[k].items()}
        out[k] = {f"{m}_us": round(t * 1000, 1) for m, t in med.items()}
        out[k].update({f"{m}_tflops": round(fl / t / 1e9, 1) for m, t in med.items()})
        print(k, json.dumps(out[k]), flush=True)
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
