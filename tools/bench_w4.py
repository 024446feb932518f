#!/usr/bin/env python3
"""4-wave persistent GEMM ("w4", gemm_bf16.hip) against the production 8-wave persistent kernel
(256n) on the BERT-base encoder shapes (M = 1024 rows x 128 tokens), plain epilogues, random data,
interleaved rounds in one process (guide §5.4 rule 24). Also checks w4 == 256n bit for bit (the
same per-element MFMA chain and epilogue arithmetic) before timing.
Usage: python tools/bench_w4.py [--rounds 5] [--iters 20]"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--M", type=int, default=131072)
    a = ap.parse_args()
    from agent_tpu_amd import ops
    from agent_tpu_amd._native import native

    nat = native()
    dev = torch.device("cuda", 0)
    M = a.M
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = {"oproj_res": (768, 768, "res"), "ffn2_res": (768, 3072, "res"), "ffn1_gelu": (3072, 768, "gelu"),
              "qkv_bias": (2304, 768, "bias")}
    cases = {}
    for name, (N, K, kind) in shapes.items():
        x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
        b = (torch.randn(N, generator=g) * 0.1).to(dev)
        r = torch.randn(M, N, generator=g).to(dev, torch.bfloat16) if kind == "res" else None
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        kw = dict(bias=b, residual=r) if kind == "res" else dict(bias=b, act="gelu") if kind == "gelu" else dict(bias=b)
        cases[name] = (x, w, kw, out, 2.0 * M * N * K)
    prev = nat.gemm_w4_mode(-1)
    ok = {}
    for name, (x, w, kw, out, _) in cases.items():
        nat.gemm_w4_mode(0)
        ref = ops.linear(x, w, **kw)
        nat.gemm_w4_mode(1)
        got = ops.linear(x, w, **kw)
        torch.cuda.synchronize()
        ok[name] = bool(torch.equal(ref, got))
        if not ok[name]:
            d = (ref.float() - got.float()).abs()
            print(json.dumps({"case": name, "mismatch": int((d > 0).sum()), "maxdiff": float(d.max())}), flush=True)
        del ref, got
    variants = {"256n": 0, "w4": 1, "w4_noepi": 2}
    res = {(n, v): [] for n in cases for v in variants}
    for _ in range(a.rounds):
        for name, (x, w, kw, out, flop) in cases.items():
            for v, mode in variants.items():
                nat.gemm_w4_mode(mode)
                ops.linear(x, w, out=out, **kw)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    ops.linear(x, w, out=out, **kw)
                e1.record()
                e1.synchronize()
                res[(name, v)].append(e0.elapsed_time(e1) * 1e3 / a.iters)
    nat.gemm_w4_mode(prev)
    for name, (_, _, _, _, flop) in cases.items():
        row = {"case": name, "exact_vs_256n": ok[name]}
        for v in variants:
            us = sorted(res[(name, v)])
            row[v + "_us"] = round(us[len(us) // 2], 1)
            row[v + "_tflops"] = round(flop / (us[len(us) // 2] * 1e-6) / 1e12, 1)
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
