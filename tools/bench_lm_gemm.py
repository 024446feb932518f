#!/usr/bin/env python3
"""Which GEMM schedule suits the decode LM-head shape? ([docs*4, d] x [V, d]^T)

Times ops.linear (bf16 output, vocab padded to a multiple of 256 so every kernel
family is eligible) with the kernel family forced (gemm_force_tile 64 / 128 / 256),
the fp32-output 128x128 form the logits path uses, the fused LM head + top-k, and
hipBLASLt (torch.mm) for reference.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agent_tpu_amd import ops  # noqa: E402
from agent_tpu_amd._native import native  # noqa: E402


def t(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    nat = native()
    dev = torch.device("cuda", 0)
    res = {}
    for name, R, V, d in (("bart", 1024, 50264, 1024), ("t5", 1024, 32128, 768)):
        Vp = (V + 255) // 256 * 256
        x = torch.randn(R, d, device=dev).bfloat16()
        w = (torch.randn(Vp, d, device=dev) * d ** -0.5).bfloat16()
        fl = 2 * R * V * d
        row = {}
        prev = nat.gemm_force_tile(-1)
        for tile in (64, 128, 256):
            nat.gemm_force_tile(tile)
            row[f"bf16_tile{tile}_us"] = round(t(lambda: ops.linear(x, w)), 1)
        nat.gemm_force_tile(prev)
        row["f32_logits_us"] = round(t(lambda: ops.linear(x, w[:V], out_f32=True)), 1)
        head = ops.LmHead(x, w[:V], None, 0.0)
        bs = torch.zeros(R, device=dev)
        row["fused_topk_us"] = round(t(lambda: head.topk(bs, 8, 2, False)), 1)
        row["hipblaslt_bf16_us"] = round(t(lambda: torch.mm(x, w.t())), 1)
        row.update({k.replace("_us", "_tflops"): round(fl / v / 1e6, 1) for k, v in list(row.items())})
        res[name] = row
        print(name, json.dumps(row), flush=True)
    print("JSON", json.dumps(res))


if __name__ == "__main__":
    main()
