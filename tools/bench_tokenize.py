#!/usr/bin/env python3
"""GPU tokenizer (K1) at the bench batch: 1024 rows of 150 synthetic words, S = 128; mean of
interleaved event-timed rounds of back-to-back launches. One JSON line."""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def main() -> int:
    from agent_tpu_amd import ops
    from agent_tpu_amd import tokenizer as T
    from agent_tpu_amd.utils.synthetic import make_text_rows

    dev = torch.device("cuda", 0)
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    text, offs = T.pack_rows(make_text_rows(rows, 150, seed=11))
    t = torch.from_numpy(text).to(dev)
    o = torch.from_numpy(offs).to(dev)
    for _ in range(5):
        ops.tokenize(t, o, 128, 30522, 2048)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ops.tokenize(t, o, 128, 30522, 2048)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000.0 / 50)
    print(json.dumps({"kernel": "tokenize", "rows": rows, "bytes": int(text.size), "us_best": round(best, 1)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
