#!/usr/bin/env python3
"""Time grouped cross attention at the summarize decode shape (docs x beams queries, encoder K/V)."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agent_tpu_amd import ops  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=256)
ap.add_argument("--beams", type=int, default=4)
ap.add_argument("--src", type=int, default=512)
ap.add_argument("--heads", type=int, default=12)
a = ap.parse_args()
dev = torch.device("cuda", 0)
H, S, nb = a.heads, a.src, a.beams
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(a.docs * nb, H * 64, generator=g, device=dev).to(torch.bfloat16)
kv = torch.randn(a.docs * S, 2 * H * 64, generator=g, device=dev).to(torch.bfloat16)
lens = torch.full((a.docs,), S, dtype=torch.int32, device=dev)
fn = lambda: ops.decode_attention(q, kv[:, :H * 64], kv[:, H * 64:], H, S, nb, lens=lens)  # noqa: E731
t = statistics.median([timeit(fn, 20) for _ in range(5)])
print(f"xattn docs={a.docs} beams={nb} S={S} H={H}: {t * 1e3:.1f} us ({kv.numel() * 2 / (t * 1e-3) / 1e12:.2f} TB/s)", flush=True)
if os.getenv("XATTN_REF"):
    red = lambda: kv.view(torch.int32).bitwise_xor_(torch.zeros(1, dtype=torch.int32, device=dev))  # noqa: E731
    t2 = statistics.median([timeit(red, 20) for _ in range(5)])
    s = lambda: torch.amax(kv, dim=0)  # noqa: E731
    t3 = statistics.median([timeit(s, 20) for _ in range(5)])
    print(f"ref: in-place xor (read+write) {kv.numel() * 4 / (t2 * 1e-3) / 1e12:.2f} TB/s, amax read "
          f"{kv.numel() * 2 / (t3 * 1e-3) / 1e12:.2f} TB/s", flush=True)
