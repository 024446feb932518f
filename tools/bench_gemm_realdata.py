#!/usr/bin/env python3
"""Why are the encoder GEMMs slower in the model than in isolation? (diagnostic)

Runs the LN-folded BERT-base encoder once on the bench's synthetic rows, captures the inputs of
layer 5's FFN1 / FFN2 / out-projection / QKV+attention calls, and times each production kernel
(interleaved rounds, back to back) on (a) those real activations and (b) random tensors of the
same shape and the same LN statistics - the data toggling changes the clock the chip holds
(MI355X_MICROARCH.md "DVFS give-back"). One JSON line per (kernel, data).
Usage: python tools/bench_gemm_realdata.py [--rows 1024]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layer", type=int, default=5)
    a = ap.parse_args()
    from agent_tpu_amd import ops
    from agent_tpu_amd.models.bert import BertClassifier, config_for, init_random
    from agent_tpu_amd.tokenizer import tokenize_rows
    from agent_tpu_amd.utils.synthetic import make_text_rows

    dev = torch.device("cuda", 0)
    cfg = config_for("bert-base")
    enc = BertClassifier(cfg, init_random(cfg, seed=0, device=dev))
    texts = [t.encode() for t in make_text_rows(a.rows, 150, seed=3)]
    ids, lens = tokenize_rows(texts, 128, cfg.vocab_size)
    ids, lens = torch.from_numpy(ids).to(dev), torch.from_numpy(lens).to(dev)
    captured = {}
    real_linear_ln, real_qkv = ops.linear_ln, ops.qkv_attention
    calls = {"n": 0}

    def cap_linear_ln(x, w, b, **kw):
        calls["n"] += 1
        key = ("ffn1" if kw.get("act") == "gelu" else "ffn2" if x.shape[1] > 1024 else
               "oproj" if kw.get("residual") is not None else "kv")
        captured.setdefault(key, []).append((x.clone(), w, b, {k: (v.clone() if torch.is_tensor(v) and k in
                                                                   ("in_fin", "res_fin", "residual") else v)
                                                                for k, v in kw.items()}))
        return real_linear_ln(x, w, b, **kw)

    def cap_qkv(x, w, b, lens_, heads, **kw):
        captured.setdefault("qkv", []).append((x.clone(), w, b, lens_, heads,
                                               {k: (v.clone() if torch.is_tensor(v) and k == "in_fin" else v)
                                                for k, v in kw.items()}))
        return real_qkv(x, w, b, lens_, heads, **kw)

    ops.linear_ln, ops.qkv_attention = cap_linear_ln, cap_qkv
    try:
        with torch.no_grad():
            enc.encode_folded(ids, lens, cls_only_last=True)
    finally:
        ops.linear_ln, ops.qkv_attention = real_linear_ln, real_qkv
    torch.cuda.synchronize()
    L = a.layer
    cands = {}

    def like(t):
        """random tensor with the real tensor's per-row mean / std (so the LN folds see the same
        statistics) and the same dtype"""
        tf = t.float()
        mu, sd = tf.mean(1, keepdim=True), tf.std(1, keepdim=True)
        return (torch.randn_like(tf) * sd + mu).to(t.dtype)

    for key in ("ffn1", "ffn2", "oproj"):
        x, w, b, kw = captured[key][L]
        out = torch.empty(x.shape[0], w.shape[0], dtype=torch.bfloat16, device=dev)
        xr = like(x)
        kw_r = dict(kw)
        if kw.get("residual") is not None:
            kw_r["residual"] = like(kw["residual"])
        for tag, xx, kk in (("real", x, kw), ("random", xr, kw_r)):
            cands[f"{key}:{tag}"] = (lambda xx=xx, w=w, b=b, kk=kk, out=out: real_linear_ln(xx, w, b, out=out, **kk))
    x, w, b, lens_, heads, kw = captured["qkv"][L]
    ctx = torch.empty(x.shape[0], w.shape[0] // 3, dtype=torch.bfloat16, device=dev)
    xr = like(x)
    cands["qkv_attn:real"] = lambda: real_qkv(x, w, b, lens_, heads, out=ctx, **kw)
    cands["qkv_attn:random"] = lambda: real_qkv(xr, w, b, lens_, heads, out=ctx, **kw)
    res = {k: [] for k in cands}
    for f in cands.values():
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
        print(json.dumps({"kernel": k, "layer": L, "us_best": round(min(v), 1), "us_all": [round(t, 1) for t in v]}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
