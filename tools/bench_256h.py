"""Persistent 256x192 GEMM (qkv_attn.hip) vs the 256x256 persistent kernel at the BERT-base
QKV shape: exactness first (both against an fp32 reference of the same op), then
interleaved timing of
  * 256s  : ops.linear_ln (the production QKV GEMM, bias | InNorm, full-line nt epilogue)
  * 256h  : gemm256h mode 0 (same math, fragment-layout stores)
  * 256h-noepi : gemm256h mode 1 (main loop only, timing only)
  * ws_*  : the wave-specialised kernel (qkv_attn_ws.hip; dev build only): attention, main loop only, Q|K|V store
Prints one JSON line per configuration. Usage: python tools/bench_256h.py [--rows 131072]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from agent_tpu_amd._native import native  # noqa: E402
from agent_tpu_amd.ops.linear import linear_ln  # noqa: E402

EPI_BIAS, EPI_IN = 1, 64


def run_h(nat, x, w, b, out, fin, col, mode):
    epi = EPI_BIAS | (EPI_IN if fin is not None else 0)
    nat.gemm256h(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0), b.data_ptr(),
                 x.shape[0], w.shape[0], x.shape[1], epi, fin.data_ptr() if fin is not None else 0,
                 col.data_ptr() if col is not None else 0, mode, torch.cuda.current_stream().cuda_stream)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="", help="comma list of kernels to time (default all)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--full-lens", action="store_true", help="every sequence 128 tokens (the bench data)")
    a = ap.parse_args()
    nat = native()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    K, N = 768, 2304
    # exactness at a small M (several persistent tiles per CU: 4096/256 * 12 = 192 tiles < 256 CUs, so
    # also 16384 rows = 768 tiles, 3 per CU)
    for M in (() if a.no_check else (4096, 16384)):
        x = (torch.randn(M, K, generator=g) * 2 + 0.3).to(torch.bfloat16).to(dev)
        w = (torch.randn(N, K, generator=g) * 0.03).to(torch.bfloat16).to(dev)
        b = (torch.randn(N, generator=g) * 0.1).to(dev)
        xf = x.float()
        mu, var = xf.mean(1), xf.var(1, unbiased=False)
        rstd = torch.rsqrt(var + 1e-12)
        fin = torch.stack([rstd, rstd * mu], 1).contiguous()
        col = w.float().sum(1).contiguous()
        for innorm in (False, True):
            ref = xf @ w.float().t()
            if innorm:
                ref = ref * fin[:, :1] - fin[:, 1:] * col.unsqueeze(0)
            ref = ref + b
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            run_h(nat, x, w, b, out, fin if innorm else None, col if innorm else None, 0)
            torch.cuda.synchronize()
            err = ((out.float() - ref).abs() / (ref.abs() + 1.0)).max().item()
            ok = err < 1.6e-2
            print(json.dumps({"check": "256h_vs_fp32", "M": M, "innorm": innorm, "max_rel_err": err, "ok": ok}),
                  flush=True)
            if not ok:
                return 1
    # timing at the bench shape
    M = a.rows
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
    b = torch.randn(N, device=dev) * 0.1
    fin = torch.stack([torch.ones(M, device=dev), torch.zeros(M, device=dev)], 1).contiguous()
    col = w.float().sum(1).contiguous()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    flop = 2.0 * M * N * K
    from agent_tpu_amd import ops

    B = M // 128
    lens = torch.randint(40, 129, (B,), device=dev, dtype=torch.int32)
    if a.full_lens:
        lens.fill_(128)
    qkv = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    ctx = torch.empty(M, N // 3, dtype=torch.bfloat16, device=dev)
    p = ops.qkv_head_order(N // 192, dev)
    w_h, b_h, col_h = w[p].contiguous(), b[p].contiguous(), col[p].contiguous()

    def unfused():
        linear_ln(x, w, b, in_fin=fin, colsum=col, out=qkv)
        ops.attention_packed(qkv, lens, B, 128, N // 192, out=ctx)

    cands = {
        "unfused_qkv_attn": unfused,
        "fused_qkv_attn": lambda: ops.qkv_attention(x, w_h, b_h, lens, N // 192, in_fin=fin, colsum_h=col_h, out=ctx),
        "256s_innorm": lambda: linear_ln(x, w, b, in_fin=fin, colsum=col, out=out),
        "256h_innorm": lambda: run_h(nat, x, w, b, out, fin, col, 0),
        "256h_noepi": lambda: run_h(nat, x, w, b, out, fin, col, 1),
        "256h_bias": lambda: run_h(nat, x, w, b, out, None, None, 0),
    }
    if a.only:
        cands = {k: f for k, f in cands.items() if k in a.only.split(",")}
    res = {k: [] for k in cands}
    for f in cands.values():
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for k, f in cands.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1000.0 / a.iters)
    for k, v in res.items():
        best = min(v)
        print(json.dumps({"kernel": k, "M": M, "N": N, "K": K, "us_best": round(best, 1),
                          "us_all": [round(t, 1) for t in v], "tflops": round(flop / best / 1e6, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
