#!/usr/bin/env python3
"""map_summarize throughput: T5-base batched beam search on one MI355X (BASELINE config 4).

Decode settings are the reference's (``/root/reference/ops/map_summarize.py:53-59``):
num_beams=4, max_length=130, min_length=30, early_stopping=True. Source docs are
synthetic text hash-tokenized to ``--src-len`` tokens (the reference truncates at
1024); weights are random-init T5-base. A step = one batch of ``--docs`` documents
summarised end to end (tokenize -> encoder -> beam-search decode -> detokenize).

Baselines (reference-shaped proxies on CPU): B12 T5-base
3.72 s/doc = 0.269 docs/s; B11 BART-large-CNN 6.47 s/doc = 0.155 docs/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

BASELINE_DOCS_PER_SEC = {"t5": 0.269, "bart": 0.155}
HBM_TBS, MFMA_PFS = 6.0, 1.3  # sustained HBM stream (MI355X_MICROARCH.md: 6.3 measured) / our GEMM main-loop rate


def roofline(cfg, docs: int, src: int, beams: int, steps: float) -> dict:
    """Bytes and FLOPs of one batch (encoder + ``steps`` decoder steps) and the time floor
    they imply: the encoder at the GEMM rate; each decoder step moves the cross K/V of every
    document (read by the beams of its item), the self K/V so far and the decoder + LM-head
    weights, and runs its projections at the GEMM rate."""
    d, f, V = cfg.d_model, cfg.d_ff, cfg.vocab_size
    Le, Ld = cfg.enc_layers, cfg.dec_layers
    rows = docs * beams
    enc_flop = docs * Le * (2 * src * (4 * d * d + 2 * d * f) + 4 * src * src * d)
    dec_flop_step = Ld * 2 * rows * (4 * d * d + 2 * d * d + 2 * d * f) + 2 * rows * d * V
    xkv_step = Ld * docs * src * 2 * d * 2
    self_kv_step = Ld * rows * (steps / 2) * 2 * d * 2
    w_step = (Ld * (6 * d * d + 2 * d * f) + V * d) * 2
    t_enc = enc_flop / (MFMA_PFS * 1e15)
    t_step = max(dec_flop_step / (MFMA_PFS * 1e15), (xkv_step + self_kv_step + w_step) / (HBM_TBS * 1e12))
    return {"encoder_tflop": round(enc_flop / 1e12, 2), "decoder_gflop_per_step": round(dec_flop_step / 1e9, 2),
            "cross_kv_mb_per_step": round(xkv_step / 1e6, 1), "self_kv_mb_per_step": round(self_kv_step / 1e6, 1),
            "decoder_weight_mb_per_step": round(w_step / 1e6, 1), "encoder_floor_ms": round(t_enc * 1e3, 2),
            "decode_floor_ms": round(t_step * steps * 1e3, 2),
            "assumes": f"{HBM_TBS} TB/s HBM, {MFMA_PFS} PF/s GEMM"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="t5-base")
    ap.add_argument("--docs", type=int, default=256, help="documents per step (batch)")
    ap.add_argument("--src-len", type=int, default=1024)  # ref truncation (ops/map_summarize.py:49)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--num-beams", type=int, default=4)
    ap.add_argument("--max-length", type=int, default=130)
    ap.add_argument("--min-length", type=int, default=30)
    ap.add_argument("--no-repeat-ngram", type=int, default=None, help="override the model default (bart-large-cnn 3)")
    a = ap.parse_args()

    from agent_tpu_amd.runtime.summarize import GenConfig, SummarizeEngine, build_model, family_of
    from agent_tpu_amd.utils.synthetic import make_text_rows

    dev = torch.device("cuda", 0)
    model, _ = build_model(a.model, device=dev, seed=0)
    eng = SummarizeEngine(model, max_source_len=a.src_len)
    gen = GenConfig(num_beams=a.num_beams, max_length=a.max_length, min_length=a.min_length,
                    no_repeat_ngram_size=a.no_repeat_ngram)
    docs = make_text_rows(a.docs * (a.warmup + a.steps), words_per_row=int(a.src_len * 0.8), seed=5)

    for w in range(a.warmup):
        eng.summarize(docs[w * a.docs:(w + 1) * a.docs], gen)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out_tokens, dec_steps = 0, 0
    tm: dict = {}
    for s in range(a.steps):
        batch = docs[(a.warmup + s) * a.docs:(a.warmup + s + 1) * a.docs]
        summaries, res = eng.summarize(batch, gen)
        out_tokens += sum(len(x) - 1 for x in res.sequences)
        dec_steps += res.steps
        for k, v in res.timing_ms.items():
            tm[k] = tm.get(k, 0.0) + v
    enc_ms, dec_ms = tm.get("encode_ms", 0.0), tm.get("decode_ms", 0.0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n = a.docs * a.steps
    print(json.dumps({
        "metric": f"summarized docs/sec map_summarize {a.model} (beams 4, max_len 130, min_len 30)",
        "value": round(n / el, 3), "unit": "docs/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(el * 1000 / a.steps, 2), "higher_is_better": True,
        "vs_baseline": round(n / el / BASELINE_DOCS_PER_SEC[family_of(a.model)], 1), "dtype": "bf16",
        "data": "synthetic text, random-init weights",
        "config": {"model": a.model, "docs_per_step": a.docs, "src_len": a.src_len, "num_beams": a.num_beams,
                   "max_length": a.max_length, "min_length": a.min_length,
                   "decode_steps_per_batch": dec_steps / a.steps,
                   "generated_tokens_per_sec": round(out_tokens / el, 1),
                   # device time between hipEvents (encoder kernels; encoder end -> last decode step)
                   "encode_ms_per_step": round(enc_ms / a.steps, 2),
                   "decode_ms_per_step": round(dec_ms / a.steps, 2),
                   "decode_ms_per_token_step": round(dec_ms / max(1, dec_steps), 3),
                   "timing_ms_per_step": {k: round(v / a.steps, 2) for k, v in sorted(tm.items())},
                   "roofline": roofline(model.cfg, a.docs, a.src_len, a.num_beams, dec_steps / a.steps)},
    }), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
