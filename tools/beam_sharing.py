#!/usr/bin/env python3
"""How much of the decode self-attention history the beams of an item share: distinct
physical cache rows per (item, key position) in the backpointer table at a few steps
(T5-base / BART, random init, graphs off so the reorder call can be observed)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import agent_tpu_amd.ops as ops  # noqa: E402
import agent_tpu_amd.runtime.summarize as sm  # noqa: E402
from agent_tpu_amd.utils.synthetic import make_text_rows  # noqa: E402

name, docs = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda", 0)
model, _ = sm.build_model(name, device=dev, seed=0)
eng = sm.SummarizeEngine(model, max_source_len=512)
seen = {}
orig = ops.beam_reorder_hist


def spy(src, dst, parent, step, last=None, off=0):
    orig(src, dst, parent, step, last=last, off=off)
    t = int(step.reshape(-1)[0])
    if last is None and t in (8, 32, 64, 96, 127):
        seen[t] = dst[:, :t + 1].cpu()


ops.beam_reorder_hist = spy
gen = sm.GenConfig(num_beams=4, max_length=130, min_length=30, use_graph=False)
eng.summarize(make_text_rows(docs, words_per_row=409, seed=5), gen)
for t, h in sorted(seen.items()):
    hh = h[:, :t].view(docs, 4, t)
    distinct = torch.tensor([[len(set(hh[b, :, j].tolist())) for j in range(t)] for b in range(docs)]).float()
    print(f"{name} step {t}: distinct rows per (item, key) mean {distinct.mean():.2f} "
          f"(1 = all 4 beams share, 4 = none); all-shared fraction {(distinct == 1).float().mean():.2f}", flush=True)
