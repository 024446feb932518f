#!/usr/bin/env python3
"""Persistent-launch prototype vs launches: the T5-base decode FFN block at
1 document x 4 beams as ONE launch with an in-launch grid barrier (ops.t5_ffn_fused) against the
two GEMV launches the decoder step runs today (RowRms|ReLU wi, K-split residual wo). Both are
captured 64x back to back in a hipGraph (the decoder step's regime) and replayed interleaved;
prints us per block for each and their agreement."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from agent_tpu_amd import ops
    from agent_tpu_amd.ops.decode import t5_ffn_fused

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    M, d, f, eps = int(os.environ.get("ROWS", "4")), 768, 3072, 1e-6
    x = (torch.randn(M, d, generator=g)).to(torch.bfloat16).to(dev)
    wi = (torch.randn(f, d, generator=g) * d ** -0.5).to(torch.bfloat16).to(dev)
    wo = (torch.randn(d, f, generator=g) * f ** -0.5).to(torch.bfloat16).to(dev)
    sync = torch.zeros(4, dtype=torch.int32, device=dev)
    hws = torch.empty(4 * f, dtype=torch.bfloat16, device=dev)

    def launches(xx):
        h = ops.linear(xx, wi, act="relu", rms_eps=eps)
        return ops.linear(h, wo, residual=xx)

    def fused(xx):
        return t5_ffn_fused(xx, wi, wo, eps, sync, h_ws=hws)

    ref = launches(x)
    out = fused(x)
    torch.cuda.synchronize()
    xf = x.float()
    hh = torch.relu(xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) @ wi.float().t())
    oracle = xf + hh.to(torch.bfloat16).float() @ wo.float().t()
    agree = {"max_abs_fused_vs_launches": (out.float() - ref.float()).abs().max().item(),
             "max_abs_fused_vs_fp32": (out.float() - oracle).abs().max().item(),
             "max_abs_launches_vs_fp32": (ref.float() - oracle).abs().max().item(),
             "sync_err_word": int(sync[2].item())}
    N = 64
    res = {}
    graphs = {}
    for name, fn in (("launches", launches), ("fused", fused)):
        xs = [x.clone() for _ in range(N + 1)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn(xs[0])
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            cur = xs[0]
            for i in range(N):  # a chain: each block's output is the next block's input
                cur = fn(cur)
        graphs[name] = gr
        res[name] = []
    for _ in range(5):
        for name, gr in graphs.items():
            gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                gr.replay()
            e1.record()
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / (10 * N))
    out = {"rows": M, "us_per_block": {k: round(sorted(v)[len(v) // 2], 3) for k, v in res.items()},
           "all_us": {k: [round(t, 3) for t in v] for k, v in res.items()}, **agree,
           "sync_err_after": int(sync[2].item())}
    out["speedup"] = round(out["us_per_block"]["launches"] / out["us_per_block"]["fused"], 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
