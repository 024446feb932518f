#!/usr/bin/env python3
"""GEMM fixed-cost ablation at the BERT-base shapes (timing only).

For each shape: full GEMM, K=64 (prologue + one K-tile + epilogue), and the
no-epilogue build (ATPU_GEMM_ABLATE=4, separate process). Prints ms and TF/s.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agent_tpu_amd import ops  # noqa: E402
from agent_tpu_amd._native import native  # noqa: E402

if os.getenv("ATPU_GEMM_ABLATE", "0") != "0":
    assert native().DEV_BUILD, "ATPU_GEMM_ABLATE needs the dev extension: python -m agent_tpu_amd.csrc.build --dev"


def t(fn, iters=30):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev = torch.device("cuda", 0)
M = 131072
g = torch.Generator(device=dev).manual_seed(0)
r = lambda *sh, sc=1.0: (torch.randn(*sh, generator=g, device=dev) * sc).to(torch.bfloat16)  # noqa: E731
x768, x3072, res = r(M, 768), r(M, 3072), r(M, 768)
shapes = {"qkv": (x768, r(2304, 768, sc=0.03), None, None), "o_res": (x768, r(768, 768, sc=0.03), None, res),
          "ffn1_gelu": (x768, r(3072, 768, sc=0.03), "gelu", None), "ffn2_res": (x3072, r(768, 3072, sc=0.03), None, res)}
out = {}
for name, (x, w, act, rr) in shapes.items():
    N, K = w.shape
    b = torch.zeros(N, dtype=torch.float32, device=dev)
    full = t(lambda: ops.linear(x, w, b, act=act, residual=rr))
    k64 = t(lambda: ops.linear(x[:, :64], w[:, :64], b, act=act, residual=rr))
    out[name] = {"full_ms": round(full, 4), "tf": round(2 * M * N * K / full / 1e9, 1), "k64_ms": round(k64, 4)}
print(json.dumps({"ablate": os.getenv("ATPU_GEMM_ABLATE", "0"), **out}))
