#!/usr/bin/env python3
"""Host-side split of a beam-search decode step: tools/host_prof_summ.py MODEL DOCS.

select = _select (includes the wait for the GPU step and the top-k D2H), to_launch = the
critical path from the selection to the next step's launch (GPU idle), after_launch =
bookkeeping overlapped with the next GPU step."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import agent_tpu_amd.runtime.summarize as sm  # noqa: E402
from agent_tpu_amd.utils.synthetic import make_text_rows  # noqa: E402

name, docs = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda", 0)
model, _ = sm.build_model(name, device=dev, seed=0)
eng = sm.SummarizeEngine(model, max_source_len=512)
gen = sm.GenConfig(num_beams=4, max_length=130, min_length=30)
rows = make_text_rows(docs * 2, words_per_row=409, seed=5)
eng.summarize(rows[:docs], gen)
torch.cuda.synchronize()
sm.HOST_PROF = {}
t = time.perf_counter()
eng.summarize(rows[docs:], gen)
torch.cuda.synchronize()
wall = time.perf_counter() - t
n = sm.HOST_PROF["steps"]
print(f"{name} docs={docs} wall {wall * 1e3:.0f} ms, {n} steps; per step: wall {wall * 1e3 / n:.2f} ms, "
      + ", ".join(f"{k} {v * 1e3 / n:.2f} ms" for k, v in sm.HOST_PROF.items() if k != "steps"))
