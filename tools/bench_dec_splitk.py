#!/usr/bin/env python3
"""Long-K decode GEMMs (M = 1024 rows): the dec kernel unsplit vs split-K (dec kernel on K slices
+ the fp32 reduce kernel), forced split counts, 50 launches per hipGraph, interleaved rounds,
median per call; outputs compared to the unsplit result. One JSON line per shape."""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agent_tpu_amd._native import native, ptr, stream_handle  # noqa: E402


def timeit(fn, iters=50):
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
    dev = torch.device("cuda", 0)
    nat = native()
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    shapes = {"t5_wo_res": (768, 3072, True, False), "t5_o_res": (768, 768, True, False),
              "t5_q": (768, 768, False, False), "bart_fc2_res": (1024, 4096, True, True),
              "bart_o_res": (1024, 1024, True, True)}
    for name, (N, K, res, has_b) in shapes.items():
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.03).bfloat16()
        b = torch.randn(N, device=dev) * 0.1 if has_b else None
        r = torch.randn(M, N, device=dev).bfloat16() if res else None
        epi = (1 if has_b else 0) | (8 if res else 0)
        ws = torch.empty(8 * M * N, dtype=torch.float32, device=dev)
        outs = {s: torch.empty(M, N, dtype=torch.bfloat16, device=dev) for s in (1, 2, 3, 4, 6)}
        t = {s: [] for s in outs}

        def run(s):
            return lambda: nat.gemm(ptr(x), K, ptr(w), K, ptr(outs[s]), N, ptr(b), ptr(r), N if res else 0, M, N, K,
                                    epi, stream_handle(), s, ptr(ws) if s > 1 else 0)
        for rd in range(4):
            for s in (list(outs) if rd % 2 == 0 else list(outs)[::-1]):
                if (K // 64) % s:
                    continue
                t[s].append(timeit(run(s)))
        rec = {"shape": name, "M": M, "N": N, "K": K}
        for s in outs:
            if t[s]:
                rec[f"split{s}_us"] = round(statistics.median(t[s]), 2)
                if s > 1:
                    rec[f"split{s}_maxdiff"] = float((outs[s].float() - outs[1].float()).abs().max())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
