#!/usr/bin/env python3
"""Decode-shaped GEMMs on the 64x64 dec kernel: 1 K-tile per barrier (4-stage ring) vs 2 K-tiles
per barrier (6-stage ring), interleaved rounds, each variant timed as 50 launches in one hipGraph;
outputs compared bit for bit. One JSON line per shape. Usage: python tools/bench_dec_kpb.py [--rows 1024]"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agent_tpu_amd import ops  # noqa: E402
from agent_tpu_amd._native import native  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1024")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    nat = native()
    shapes = {  # name: (N, K, act, residual)
        "t5_qkv": (2304, 768, None, False), "t5_o_res": (768, 768, None, True), "t5_q": (768, 768, None, False),
        "t5_wi_relu": (3072, 768, "relu", False), "t5_wo_res": (768, 3072, None, True),
        "bart_o_res": (1024, 1024, None, True), "bart_fc1_gelu": (4096, 1024, "gelu", False),
        "bart_fc2_res": (1024, 4096, None, True),
    }
    for M in [int(x) for x in a.rows.split(",")]:
        for name, (N, K, act, res) in shapes.items():
            x = torch.randn(M, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) * 0.03).bfloat16()
            b = torch.randn(N, device=dev) * 0.1
            r = torch.randn(M, N, device=dev).bfloat16() if res else None
            y = {1: torch.empty(M, N, device=dev, dtype=torch.bfloat16),
                 2: torch.empty(M, N, device=dev, dtype=torch.bfloat16)}
            t = {1: [], 2: []}
            for rd in range(a.rounds):
                for kpb in ((1, 2) if rd % 2 == 0 else (2, 1)):
                    nat.gemm_dec_kpb(kpb)
                    t[kpb].append(timeit(lambda: ops.linear(x, w, b, act=act, residual=r, out=y[kpb]), a.iters))
            nat.gemm_dec_kpb(1)
            u1, u2 = statistics.median(t[1]), statistics.median(t[2])
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "kpb1_us": round(u1, 2), "kpb2_us": round(u2, 2),
                              "speedup": round(u1 / u2, 3), "bit_identical": bool(torch.equal(y[1], y[2]))}),
                  flush=True)


if __name__ == "__main__":
    main()
