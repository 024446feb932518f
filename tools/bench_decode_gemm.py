#!/usr/bin/env python3
"""Decode-shaped GEMMs (M = docs x beams): 64x64 multi-stage dec kernel vs the
128x128 split-K path, per T5-base / BART-large decoder projection, hipEvent
timing over back-to-back launches, interleaved rounds, median reported."""
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
from agent_tpu_amd.ops.linear import _splits  # noqa: E402


def timeit(fn, iters):
    """GPU time per call: ``iters`` calls captured in one hipGraph (no host gaps)."""
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
    ap.add_argument("--rows", default="256,1024")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    shapes = {  # name: (N, K, act, residual)
        "t5_qkv": (2304, 768, None, False), "t5_o_res": (768, 768, None, True), "t5_q": (768, 768, None, False),
        "t5_wi_relu": (3072, 768, "relu", False), "t5_wo_res": (768, 3072, None, True),
        "bart_qkv": (3072, 1024, None, False), "bart_o_res": (1024, 1024, None, True),
        "bart_fc1_gelu": (4096, 1024, "gelu", False), "bart_fc2_res": (1024, 4096, None, True),
    }
    out = {}
    for M in [int(x) for x in a.rows.split(",")]:
        for name, (N, K, act, res) in shapes.items():
            x = torch.randn(M, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) * 0.03).bfloat16()
            b = torch.randn(N, device=dev) * 0.1 if name.startswith("bart") else None  # T5: no biases
            r = torch.randn(M, N, device=dev).bfloat16() if res else None
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            t = {0: [], 1: []}
            for rd in range(a.rounds):
                for mode in ((0, 1) if rd % 2 == 0 else (1, 0)):
                    native().gemm_dec_mode(mode)
                    _splits.cache_clear()
                    t[mode].append(timeit(lambda: ops.linear(x, w, b, act=act, residual=r, out=y), a.iters))
            # dec kernel without split-K (explicit splits=1 through the binding)
            from agent_tpu_amd._native import ptr, stream_handle
            epi = (1 if b is not None else 0) | {None: 0, "gelu": 2, "relu": 16}[act] | (8 if res else 0)
            native().gemm_dec_mode(1)
            t_ns = statistics.median(timeit(lambda: native().gemm(
                ptr(x), K, ptr(w), K, ptr(y), N, ptr(b), ptr(r), N if res else 0, M, N, K, epi, stream_handle(),
                1, 0), a.iters) for _ in range(a.rounds))
            _splits.cache_clear()
            ref = ops.linear(x, w, b, act=act, residual=r)
            native().gemm_dec_mode(0)
            _splits.cache_clear()
            old = ops.linear(x, w, b, act=act, residual=r)
            native().gemm_dec_mode(1)
            _splits.cache_clear()
            err = ((ref.float() - old.float()).abs().max() / old.float().abs().max()).item()
            us0, us1 = statistics.median(t[0]), statistics.median(t[1])
            fl = 2.0 * M * N * K
            out[f"{name}_M{M}"] = {"splitk128_us": round(us0, 2), "dec_us": round(us1, 2),
                                   "speedup": round(us0 / us1, 2), "dec_tflops": round(fl / us1 / 1e6, 1),
                                   "dec_splits": _splits(M, N, K), "dec_nosplit_us": round(t_ns, 2),
                                   "rel_diff": err}
            print(f"{name}_M{M}", json.dumps(out[f"{name}_M{M}"]), flush=True)
    print("JSON " + json.dumps(out))


if __name__ == "__main__":
    main()
