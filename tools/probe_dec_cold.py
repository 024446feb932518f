#!/usr/bin/env python3
"""Decode GEMMs (M = 1024 rows: 256 docs x 4 beams) with hot weights (back to back) vs cold
weights (L2 and MALL flushed by a 1 GiB stream before each call, as the cross-attention K/V
stream does between a decode step's GEMMs): is the in-model slowdown the weights' first fetch?
Event-timed per call. One JSON line per shape."""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agent_tpu_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M = 1024
    flush_src = torch.empty(1 << 29, dtype=torch.float16, device=dev).normal_()  # 1 GiB
    flush_dst = torch.empty_like(flush_src)
    shapes = {"t5_qkv": (2304, 768, None, False), "t5_o_res": (768, 768, None, True), "t5_q": (768, 768, None, False),
              "t5_wi_relu": (3072, 768, "relu", False), "t5_wo_res": (768, 3072, None, True),
              "bart_fc1_gelu": (4096, 1024, "gelu", False), "bart_fc2_res": (1024, 4096, None, True)}
    for name, (N, K, act, res) in shapes.items():
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.03).bfloat16()
        b = torch.randn(N, device=dev) * 0.1 if name.startswith("bart") else None  # T5: no biases
        r = torch.randn(M, N, device=dev).bfloat16() if res else None
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        f = lambda: ops.linear(x, w, b, act=act, residual=r, out=y)
        out = {}
        for mode in ("hot", "cold", "hot", "cold"):
            ts = []
            for _ in range(30):
                if mode == "cold":
                    flush_dst.copy_(flush_src)
                else:
                    f()
                torch.cuda._sleep(2_000_000)  # the GPU busy while the host enqueues: no launch gap timed
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000.0)
            out.setdefault(mode, []).append(statistics.median(ts))
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "hot_us": round(min(out["hot"]), 2),
                          "cold_us": round(min(out["cold"]), 2)}), flush=True)


if __name__ == "__main__":
    main()
