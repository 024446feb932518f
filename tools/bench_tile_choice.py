#!/usr/bin/env python3
"""GEMM kernel family per decode-shaped problem: auto choice vs forced dec (64x64) / 128x128 / 256x256,
graph-timed (tools/bench_decode_gemm.timeit), T5-base and BART-large decoder projections at several M."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agent_tpu_amd import ops  # noqa: E402
from agent_tpu_amd._native import native  # noqa: E402
from tools.bench_decode_gemm import timeit  # noqa: E402

nat = native()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
shapes = {"t5_qkv": (2304, 768, None, False), "t5_o_res": (768, 768, None, True), "t5_wi_relu": (3072, 768, "relu", False),
          "t5_wo_res": (768, 3072, None, True), "bart_qkv": (3072, 1024, None, False),
          "bart_o_res": (1024, 1024, None, True), "bart_fc1_gelu": (4096, 1024, "gelu", False),
          "bart_fc2_res": (1024, 4096, None, True)}
rows = [int(v) for v in os.environ.get("ROWS", "1024,2048,4096").split(",")]
for M in rows:
    for name, (N, K, act, res) in shapes.items():
        x = torch.randn(M, K, generator=g, device=dev).bfloat16()
        w = (torch.randn(N, K, generator=g, device=dev) * 0.03).bfloat16()
        r = torch.randn(M, N, generator=g, device=dev).bfloat16() if res else None
        out = {}
        for mode in (0, 64, 128, 256):
            nat.gemm_force_tile(mode)
            try:
                ops.linear.__globals__["_splits"].cache_clear()
                out[mode] = statistics.median(timeit(lambda: ops.linear(x, w, act=act, residual=r), 20) for _ in range(3))
            except Exception as e:  # noqa: BLE001
                out[mode] = float("nan")
        nat.gemm_force_tile(0)
        ops.linear.__globals__["_splits"].cache_clear()
        print(f"{name} M={M}", json.dumps({f"{'auto' if k == 0 else k}_us": round(v, 2) for k, v in out.items()}), flush=True)
