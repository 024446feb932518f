"""How much of a 4-row decode GEMV is weight-load latency? Times ops.linear at M = 4 on
  * hot  : the same weight matrix every call (L2-resident after the first)
  * mall : a ring of matrices that fits the Infinity Cache but not L2
  * cold : a ring larger than the Infinity Cache (HBM)
for the T5-base decoder shapes. One JSON line per (shape, mode)."""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from agent_tpu_amd import ops  # noqa: E402


def main() -> int:
    dev = torch.device("cuda", 0)
    for (N, K, act) in ((768, 768, None), (3072, 768, "relu"), (768, 3072, None), (2304, 768, None)):
        mb = N * K * 2 / 2**20
        x = torch.randn(4, K, device=dev).to(torch.bfloat16)
        for mode, ring_mb in (("hot", 0), ("mall", 96), ("cold", 1024)):
            n = max(1, int(ring_mb / mb)) if ring_mb else 1
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(n)]
            out = torch.empty(4, N, device=dev, dtype=torch.bfloat16)
            for i in range(3 * n):
                ops.linear(x, ws[i % n], act=act, out=out)
            torch.cuda.synchronize()
            iters = max(200, 2 * n)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(iters):
                    ops.linear(x, ws[i % n], act=act, out=out)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1000 / iters
            print(json.dumps({"N": N, "K": K, "weights_mb": round(mb, 2), "mode": mode, "ring": n,
                              "us_per_gemv_in_graph": round(us, 2)}), flush=True)
            del ws, g
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
