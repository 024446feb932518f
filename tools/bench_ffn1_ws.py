#!/usr/bin/env python3
"""BERT-base FFN1 (M x 768 -> 3072, LN-folded input, bias, GELU): the 256 x 256 production
kernel (ops.linear_ln) against the wave-specialised kernel (ops.linear.gemm_ws), interleaved
rounds on random data; also the ws main loop alone (timing only) and the plain (no GELU) form.
One JSON line per configuration. Needs a dev build of the extension (build.py --dev: the ws kernels
are not in the release build). Usage: python tools/bench_ffn1_ws.py [--rows 131072] [--variants 8,24]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from agent_tpu_amd._native import native  # noqa: E402
from agent_tpu_amd.ops.linear import gemm_ws, linear_ln  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--n", type=int, default=3072)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="8,72,104")
    a = ap.parse_args()
    nat = native()
    dev = torch.device("cuda", 0)
    M, K, N = a.rows, 768, a.n
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
    b = torch.randn(N, device=dev) * 0.1
    xf = x.float()
    rstd = torch.rsqrt(xf.var(1, unbiased=False) + 1e-12)
    fin = torch.stack([rstd, rstd * xf.mean(1)], 1).contiguous()
    del xf
    col = w.float().sum(1).contiguous()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)

    def ws(var, **kw):
        def run():
            nat.ws_variant(var)
            gemm_ws(x, w, b, out, in_fin=fin, colsum=col, **kw)
        return run

    cands = {"256s_ffn1": lambda: linear_ln(x, w, b, act="gelu", in_fin=fin, colsum=col, out=out)}
    for var in [int(v) for v in a.variants.split(",")]:
        cands[f"ws_ffn1@{var}"] = ws(var, gelu=True)
        cands[f"ws_plain@{var}"] = ws(var, gelu=False)
        cands[f"ws_noepi@{var}"] = ws(var, gelu=False, timing_only=True)
    res = {k: [] for k in cands}
    for f in cands.values():
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for k, f in cands.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1000.0 / a.iters)
    flop = 2.0 * M * N * K
    for k, v in res.items():
        best = min(v)
        print(json.dumps({"kernel": k, "M": M, "N": N, "K": K, "us_best": round(best, 1),
                          "us_all": [round(t, 1) for t in v], "tflops": round(flop / best / 1e6, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
