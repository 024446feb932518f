#!/usr/bin/env python3
"""Time the fused log-softmax + beam top-k kernel at the T5 decode shape (rows x vocab fp32 logits)."""
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
ap.add_argument("--vocab", type=int, default=32128)
ap.add_argument("--k", default="8,9")
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
logits = torch.randn(a.rows, a.vocab, generator=g, device=dev) * 3
bs = torch.randn(a.rows, generator=g, device=dev)
for k in [int(v) for v in a.k.split(",")]:
    t = [timeit(lambda: ops.beam_topk_rows(logits, bs, k, eos=1, mask_eos=True), 20) for _ in range(5)]
    print(f"k={k} rows={a.rows} V={a.vocab}: {statistics.median(t) * 1000:.1f} us "
          f"({a.rows * a.vocab * 4 / statistics.median(t) / 1e9:.2f} TB/s)", flush=True)
