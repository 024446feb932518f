#!/usr/bin/env python3
"""Summarize stage clocks vs the kernels: ``encode_ms`` from the hipEvent
pair in generate() against (a) the same encoder replayed alone and timed by events around it,
and (b) under ``rocprofv3 --kernel-trace --stats`` with ``--encode-only``, the kernel-time sum
of those encoder calls. Prints one JSON line."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="t5-base")
    ap.add_argument("--docs", type=int, default=256)
    ap.add_argument("--src-len", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--encode-only", action="store_true")
    a = ap.parse_args()
    from agent_tpu_amd.runtime.summarize import GenConfig, SummarizeEngine, build_model
    from agent_tpu_amd.utils.synthetic import make_text_rows

    dev = torch.device("cuda", 0)
    model, _ = build_model(a.model, device=dev, seed=0)
    eng = SummarizeEngine(model, max_source_len=a.src_len)
    docs = make_text_rows(a.docs, words_per_row=int(a.src_len * 0.8), seed=5)
    ids, lens, _ = eng.encode_texts(docs, with_maps=False)
    out = {"model": a.model, "docs": a.docs, "src_len": int(ids.shape[1])}
    if not a.encode_only:
        gen = GenConfig(num_beams=4, max_length=130, min_length=30)
        eng.summarize(docs, gen)  # warm-up (graphs, caches)
        enc = []
        for _ in range(a.reps):
            _, res = eng.summarize(docs, gen)
            enc.append(res.timing_ms["encode_ms"])
        out["generate_encode_ms"] = [round(x, 2) for x in enc]
        out["generate_timing_ms"] = {k: round(v, 2) for k, v in res.timing_ms.items()}
    model.encode(ids, lens)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    alone = []
    for _ in range(a.reps):
        e0.record()
        model.encode(ids, lens)
        e1.record()
        e1.synchronize()
        alone.append(e0.elapsed_time(e1))
    out["encode_alone_ms"] = [round(x, 2) for x in alone]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
