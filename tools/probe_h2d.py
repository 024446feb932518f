#!/usr/bin/env python3
"""Host -> HBM upload of a model-sized byte buffer, by method (weights upload, C1 source).

Prints ms and GB/s (best of 3) for a 219 MB (BERT-base bf16) pageable buffer: plain
pageable .to(), pin_memory() + async copy, and a copy from an already pinned buffer (the
DMA floor). Round 4 measured pageable 56 GB/s = pinned 57.5 (and a two-slot pinned
staging in 32 MiB chunks 40 GB/s, since removed): ParamPack.to stays a plain copy
(profiles/h2d_upload_r04.json)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def main():
    dev = torch.device("cuda", 0)
    torch.empty(1, device=dev)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 219_212_032
    src = torch.randint(0, 256, (n,), dtype=torch.uint8)
    pinned = src.pin_memory()
    res = {"bytes": n, "torch_threads": torch.get_num_threads()}
    res["pageable_to"] = timed(lambda: src.to(dev))
    res["pin_then_copy"] = timed(lambda: src.pin_memory().to(dev, non_blocking=True))
    res["from_pinned"] = timed(lambda: pinned.to(dev, non_blocking=True))
    out = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}
    out.update({k + "_GBps": round(n / v / 1e6, 1) for k, v in res.items() if isinstance(v, float)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
