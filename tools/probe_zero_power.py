"""Does an MFMA-bound GEMM run faster on zeros? (PERF_NOTES "Producer GEMM finalizing ...")

Times the encoder's FFN1 shape (ops.linear, 65536 x 3072 x 768, bias + GELU) back to back on
random bf16 data and on all-zero activations, alternating, and prints one JSON line per round.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agent_tpu_amd import ops


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    dev = "cuda"
    M, K, N = 65536, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((M, K), generator=g, device=dev).to(torch.bfloat16)
    z = torch.zeros_like(x)
    w = (0.02 * torch.randn((N, K), generator=g, device=dev)).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    out = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    for a in (x, z):
        timed(lambda: ops.linear(a, w, b, act="gelu", out=out), 20)
    for rnd in range(3):
        tr = timed(lambda: ops.linear(x, w, b, act="gelu", out=out), 200)
        tz = timed(lambda: ops.linear(z, w, b, act="gelu", out=out), 200)
        print(json.dumps({"round": rnd, "random_us": round(tr, 1), "zeros_us": round(tz, 1),
                          "zeros_speedup": round(tr / tz, 3)}), flush=True)


if __name__ == "__main__":
    main()
