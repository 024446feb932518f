#!/usr/bin/env python3
"""Decode GEMMs with the RMSNorm folded in (kEpiRowRms) vs the plain GEMM, T5-base shapes, graph-timed."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agent_tpu_amd import ops  # noqa: E402
from tools.bench_decode_gemm import timeit  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
M = int(os.environ.get("ROWS", "1024"))
x = torch.randn(M, 768, generator=g, device=dev).bfloat16()
for name, N, act in (("qkv", 2304, None), ("cq", 768, None), ("wi_relu", 3072, "relu"), ("lm_f32", 32128, None)):
    w = (torch.randn(N, 768, generator=g, device=dev) * 0.03).bfloat16()
    f32 = name == "lm_f32"
    plain = [timeit(lambda: ops.linear(x, w, act=act, out_f32=f32), 30) for _ in range(3)]
    rms = [timeit(lambda: ops.linear(x, w, act=act, out_f32=f32, rms_eps=1e-6), 30) for _ in range(3)]
    print(f"{name} M={M}: plain {statistics.median(plain):.2f} us, rms-folded {statistics.median(rms):.2f} us", flush=True)
