#!/usr/bin/env python3
"""Per-kernel microbenchmarks at the BERT-base S=128 shapes (random data).

Interleaved rounds in one process (guide §5.4 rule 24): each variant is timed
with hipEvents over `iters` launches, the round order alternates, and the
median is reported. Compares the hand-written kernels against the library
(hipBLASLt via torch.matmul, torch SDPA) on identical inputs.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agent_tpu_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--docs", type=int, default=256, help="long-sequence attention cases: documents")
    ap.add_argument("--src", type=int, default=1024, help="long-sequence attention cases: tokens per document")
    ap.add_argument("--variants", default="",
                    help="comma list of extra 256x256 GEMM variants to time (0=256b, 2=256p+nt stores)")
    a = ap.parse_args()
    from agent_tpu_amd._native import native

    nat = native()
    dev = torch.device("cuda", 0)
    M = a.rows * 128
    H, I = 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*shape, scale=1.0, dtype=torch.bfloat16):
        return (torch.randn(*shape, generator=g, device=dev) * scale).to(dtype)

    x768, x3072 = r(M, H), r(M, I)
    wqkv, wo, w1, w2 = r(3 * H, H, scale=0.03), r(H, H, scale=0.03), r(I, H, scale=0.03), r(H, I, scale=0.03)
    bqkv, bo, b1, b2 = (r(n, scale=0.1, dtype=torch.float32) for n in (3 * H, H, I, H))
    res = r(M, H)
    out = {}
    cases = {
        "gemm_qkv": (lambda: ops.linear(x768, wqkv, bqkv), lambda: torch.addmm(bqkv.bfloat16(), x768, wqkv.t()),
                     2 * M * H * 3 * H),
        "gemm_o_res": (lambda: ops.linear(x768, wo, bo, residual=res),
                       lambda: torch.addmm(bo.bfloat16(), x768, wo.t()).add_(res), 2 * M * H * H),
        "gemm_ffn1_gelu": (lambda: ops.linear(x768, w1, b1, act="gelu"),
                           lambda: torch.nn.functional.gelu(torch.addmm(b1.bfloat16(), x768, w1.t())), 2 * M * H * I),
        "gemm_ffn2_res": (lambda: ops.linear(x3072, w2, b2, residual=res),
                          lambda: torch.addmm(b2.bfloat16(), x3072, w2.t()).add_(res), 2 * M * I * H),
    }
    extra = {}  # per case: name -> extra timed callable
    qkv = r(M, 3 * H)
    lens = torch.full((a.rows,), 128, dtype=torch.int32, device=dev)
    q4 = qkv[:, :H].view(a.rows, 128, 12, 64).transpose(1, 2)
    k4 = qkv[:, H:2 * H].view(a.rows, 128, 12, 64).transpose(1, 2)
    v4 = qkv[:, 2 * H:].view(a.rows, 128, 12, 64).transpose(1, 2)
    cases["attention"] = (lambda: ops.attention_packed(qkv, lens, a.rows, 128, 12),
                          lambda: torch.nn.functional.scaled_dot_product_attention(q4, k4, v4),
                          4 * a.rows * 12 * 128 * 128 * 64)
    if any(k.startswith("attn_flash") for k in a.only.split(",")):
        # summarizer encoder attention at the reference's source length (flash kernel): T5 with the
        # relative-position bias by distance, BART without bias; library = torch SDPA (dense bias mask)
        D_, S_ = a.docs, a.src
        ql, kl, vl = r(D_ * S_, H), r(D_ * S_, H), r(D_ * S_, H)
        lens_l = torch.full((D_,), S_, dtype=torch.int32, device=dev)
        bd = r(12, 2 * S_ - 1, dtype=torch.float32)
        from agent_tpu_amd.ops.attention import dist_to_dense

        dense = dist_to_dense(bd, S_, S_).unsqueeze(0).bfloat16()
        qs, ks, vs = (t.view(D_, S_, 12, 64).transpose(1, 2) for t in (ql, kl, vl))
        fl_l = 4 * D_ * 12 * S_ * S_ * 64
        cases["attn_flash_t5"] = (lambda: ops.attention(ql, kl, vl, lens_l, D_, S_, S_, 12, scale=1.0, bias_dist=bd),
                                  lambda: torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, attn_mask=dense,
                                                                                           scale=1.0), fl_l)
        cases["attn_flash_bart"] = (lambda: ops.attention(ql, kl, vl, lens_l, D_, S_, S_, 12),
                                    lambda: torch.nn.functional.scaled_dot_product_attention(qs, ks, vs), fl_l)
    if any(k.startswith("lm_") for k in a.only.split(",")):
        # decode LM head at --docs x 4 beam rows: fused GEMM + top-k (lm_head.hip) against the
        # fp32-logit GEMM + beam_topk_rows pair it replaces ("lib" here = that pair)
        for name, V_, d_, rms in (("lm_bart", 50264, 1024, False), ("lm_t5", 32128, 768, True)):
            R_ = a.docs * 4
            head = ops.LmHead(r(R_, d_), r(V_, d_, scale=d_ ** -0.5),
                              None if rms else r(V_, scale=0.5, dtype=torch.float32), 1e-6 if rms else 0.0)
            bsc = torch.zeros(R_, device=dev)
            cases[name] = (lambda h=head, b=bsc: h.topk(b, 8, 2, False),
                           lambda h=head, b=bsc: ops.beam_topk_rows(h.logits(), b, 8, 2, False), 2 * R_ * V_ * d_)
            extra[name] = {"gemm_only": lambda h=head: h.logits()}
    gam, bet = r(H, dtype=torch.float32), r(H, dtype=torch.float32)
    cases["layernorm"] = (lambda: ops.layernorm(x768, gam, bet, 1e-12),
                          lambda: torch.nn.functional.layer_norm(x768, (H,), gam.bfloat16(), bet.bfloat16(), 1e-12),
                          0)
    sel = [k for k in cases if not a.only or k in a.only.split(",")]
    variants = [int(v) for v in a.variants.split(",") if v]
    times = {k: {"ours": [], "lib": [], "p16": [], **{f"cfg{c}": [] for c in range(6)}, **{f"v{v}": [] for v in variants},
                 **{e: [] for e in extra.get(k, {})}} for k in sel}
    prev_var = nat.gemm_256_variant(-1)
    for rd in range(a.rounds):
        for k in (sel if rd % 2 == 0 else list(reversed(sel))):
            ours, lib, _ = cases[k]
            times[k]["ours"].append(timeit(ours, a.iters))
            times[k]["lib"].append(timeit(lib, a.iters))
            if k.startswith("gemm"):
                for v in variants:
                    nat.gemm_256_variant(v)
                    times[k][f"v{v}"].append(timeit(ours, a.iters))
                    nat.gemm_256_variant(prev_var)
            for e, fn in extra.get(k, {}).items():
                times[k][e].append(timeit(fn, a.iters))
            if k.startswith("lm_"):  # A/B: tile / LDS ring / wave-grid configs (lm_head.hip; dev build)
                prev = nat.lm_head_stages(-1)
                for c in range(6):
                    nat.lm_head_stages(c)
                    times[k][f"cfg{c}"].append(timeit(ours, a.iters))
                nat.lm_head_stages(prev)
            if k == "attention":  # A/B: the 16-query persistent kernel (mode 1)
                prev = nat.attention_persist_mode(-1)
                nat.attention_persist_mode(1)
                times[k]["p16"].append(timeit(ours, a.iters))
                nat.attention_persist_mode(prev)
    for k in sel:
        fl = cases[k][2]
        o, l = statistics.median(times[k]["ours"]), statistics.median(times[k]["lib"])
        out[k] = {"ours_ms": round(o, 4), "lib_ms": round(l, 4), "speedup_vs_lib": round(l / o, 3)}
        if fl:
            out[k]["ours_tflops"] = round(fl / o / 1e9, 1)
            out[k]["lib_tflops"] = round(fl / l / 1e9, 1)
        for e in [f"cfg{c}" for c in range(6)] + list(extra.get(k, {})):
            if times[k][e]:
                out[k][f"{e}_ms"] = round(statistics.median(times[k][e]), 4)
        if times[k]["p16"]:
            out[k]["p16_ms"] = round(statistics.median(times[k]["p16"]), 4)
        for v in variants:
            if times[k][f"v{v}"]:
                out[k][f"v{v}_tflops"] = round(fl / statistics.median(times[k][f"v{v}"]) / 1e9, 1)
        print(k, json.dumps(out[k]), flush=True)
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
