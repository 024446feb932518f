#!/usr/bin/env python3
"""Fused LM head + beam top-k at few rows (a 1-document decode step: 4 rows): per-call time of
ops.lm_head_topk (main kernel + merge, + the ban bitmap for BART) for every LM-head
configuration the build has (ATPU_LM_CFG: release builds run 0 only), T5-base and
BART-large-CNN shapes, 50 calls per hipGraph, median of interleaved rounds. One JSON line
per (model, rows, cfg)."""
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
from tools.bench_dec_splitk import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[4, 16])
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    nat = native()
    cfgs = [0]
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = {"t5-base": (32128, 768, True, False), "bart-large-cnn": (50264, 1024, False, True)}
    for model, (V, d, rms, has_bias) in shapes.items():
        w = (torch.randn(V, d, generator=g) / d ** 0.5).to(dev, torch.bfloat16)
        b = (torch.randn(V, generator=g) * 0.5).to(dev) if has_bias else None
        for R in a.rows:
            x = torch.randn(R, d, generator=g).to(dev, torch.bfloat16)
            bs = torch.randn(R, generator=g).to(dev)
            bans = torch.full((R, 4), -1, dtype=torch.int32, device=dev) if has_bias else None
            t = {c: [] for c in cfgs}
            for rd in range(a.rounds):
                for c in (cfgs if rd % 2 == 0 else cfgs[::-1]):
                    nat.lm_head_stages(c)
                    t[c].append(timeit(lambda: ops.lm_head_topk(x, w, bs, 8, 1, True, bias=b,
                                                                rms_eps=1e-6 if rms else 0.0, bans=bans)))
            nat.lm_head_stages(0)
            for c in cfgs:
                print(json.dumps({"model": model, "rows": R, "V": V, "d": d, "cfg": c,
                                  "us_per_call": round(statistics.median(t[c]), 2)}), flush=True)


if __name__ == "__main__":
    main()
