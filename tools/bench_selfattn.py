#!/usr/bin/env python3
"""Time the decode self-attention (all heads per row) at the summarize shape under three
backpointer patterns: every beam reads its item's beam-0 rows (shared prefix), its own rows,
or random rows."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agent_tpu_amd import ops  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1024)
ap.add_argument("--heads", type=int, default=12)
ap.add_argument("--T", type=int, default=130)
ap.add_argument("--t", type=int, default=65)
a = ap.parse_args()
dev = torch.device("cuda", 0)
R, H, T, d = a.rows, a.heads, a.T, a.heads * 64
g = torch.Generator(device=dev).manual_seed(0)
cache = torch.randn(R * T, 2 * d, generator=g, device=dev).to(torch.bfloat16)
q = torch.randn(R, 3 * d, generator=g, device=dev).to(torch.bfloat16)[:, :d]
step = torch.tensor([a.t], dtype=torch.int32, device=dev)
bias = torch.randn(H, T, generator=g, device=dev)
pats = {
    "shared": (torch.arange(R, device=dev) // 4 * 4).view(-1, 1).expand(R, T),
    "own": torch.arange(R, device=dev).view(-1, 1).expand(R, T),
    "random": torch.randint(0, R, (R, T), generator=g, device=dev),
}
for name, h in pats.items():
    hist = h.to(torch.int32).contiguous()
    fn = lambda: ops.decode_attention(q, cache[:, :d], cache[:, d:], H, T, 1, step=step, bias_dist=bias,  # noqa: E731
                                      hist=hist)
    t = statistics.median([timeit(fn, 20) for _ in range(5)])
    kv = R * (a.t + 1) * d * 2 * 2
    print(f"self-attn rows={R} H={H} t={a.t} {name}: {t * 1e3:.1f} us ({kv / (t * 1e-3) / 1e12:.2f} TB/s logical)",
          flush=True)
