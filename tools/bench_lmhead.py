#!/usr/bin/env python3
"""LM-head GEMM (fp32 logits, RMSNorm folded / plain) per kernel family, graph-timed."""
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
for (V, d, rms) in ((32128, 768, True), (50264, 1024, False)):
    w = (torch.randn(V, d, generator=g, device=dev) * 0.03).bfloat16()
    b = None if rms else torch.randn(V, generator=g, device=dev) * 0.1
    for M in (1024, 4096):
        x = torch.randn(M, d, generator=g, device=dev).bfloat16()
        res = {}
        for mode in (0, 64, 128):
            nat.gemm_force_tile(mode)
            f = lambda: ops.linear(x, w, b, out_f32=True, rms_eps=1e-6 if rms else None)  # noqa: E731
            res[mode] = statistics.median(timeit(f, 10) for _ in range(3))
        nat.gemm_force_tile(0)
        fl = 2 * M * V * d
        print(f"V={V} d={d} M={M} rms={rms}: " + ", ".join(f"{k or 'auto'} {v:.1f} us ({fl / v / 1e6:.0f} TF/s)"
                                                            for k, v in res.items()), flush=True)
