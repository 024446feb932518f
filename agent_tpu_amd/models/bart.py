"""BART encoder-decoder on the gfx950 kernels (map_summarize, family ``bart``).

The reference summarizer is HF ``facebook/bart-large-cnn`` run through
``BartForConditionalGeneration.generate`` on the CPU
(``/root/reference/ops/map_summarize.py:9,46-59``). Same graph here, on the
kernels the BERT path already uses (BART's post-LN layer has BERT's shape):

  encoder : embed + learned positions (offset 2) + LayerNorm (K2)
            -> L x [fused QKV GEMM + bias, attention (K4, 1/sqrt(64)),
                    O-proj + bias + residual (GEMM epilogue), LayerNorm,
                    FC1 + bias + GELU (epilogue), FC2 + bias + residual, LN]
            -> ONE GEMM producing every decoder layer's cross K|V (+ bias).
  decoder : per generated token: embed + position row of the device step + LN,
            L x [QKV GEMM, KV-cache append, single-query self attention over
                 the beam-backpointer history (K9), O-proj + residual, LN,
                 cross Q GEMM, grouped cross attention over the item's encoder
                 K/V, O-proj + residual, LN, FC1 GELU, FC2 + residual, LN]
            -> tied LM head + final_logits_bias with fp32 logits (K10 input).

Parameter layout follows HF ``BartForConditionalGeneration`` (Linear weights
``[out, in]``), so :func:`from_hf_state_dict` is a rename + concat.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from .. import ops
from .params import ParamPack, rand_fill

POS_OFFSET = 2  # BartLearnedPositionalEmbedding offset


@dataclass(frozen=True)
class BartConfig:
    vocab_size: int = 50264
    d_model: int = 1024
    heads: int = 16
    d_ff: int = 4096
    enc_layers: int = 12
    dec_layers: int = 12
    max_positions: int = 1024
    eps: float = 1e-5
    pad_id: int = 1
    bos_id: int = 0
    eos_id: int = 2
    decoder_start_id: int = 2
    # generation defaults of facebook/bart-large-cnn's generation_config (the
    # reference's generate() call overrides only beams/max/min/early_stopping)
    forced_bos_id: Optional[int] = 0
    forced_eos_id: Optional[int] = 2
    no_repeat_ngram_size: int = 3
    length_penalty: float = 2.0

    def param_count(self) -> int:
        d, f = self.d_model, self.d_ff
        enc = self.enc_layers * (4 * d * d + 2 * d * f + 9 * d + f)
        dec = self.dec_layers * (8 * d * d + 2 * d * f + 15 * d + f)
        return self.vocab_size * (d + 1) + 2 * (self.max_positions + POS_OFFSET) * d + 4 * d + enc + dec


PRESETS: Dict[str, BartConfig] = {
    "bart-large-cnn": BartConfig(),
    "bart-large": BartConfig(no_repeat_ngram_size=0, length_penalty=1.0, forced_bos_id=None),
    "bart-base": BartConfig(d_model=768, heads=12, d_ff=3072, enc_layers=6, dec_layers=6),
    "bart-tiny": BartConfig(vocab_size=4096, d_model=256, heads=4, d_ff=512, enc_layers=2, dec_layers=2,
                            max_positions=256),
}


def config_for(name: str, **overrides) -> BartConfig:
    key = name.split("/")[-1]  # accept "facebook/bart-large-cnn"
    if key not in PRESETS:
        raise ValueError(f"unknown BART preset {name!r}; known: {sorted(PRESETS)}")
    return dataclasses.replace(PRESETS[key], **overrides)


def param_specs(cfg: BartConfig):
    d, f, bf, f32 = cfg.d_model, cfg.d_ff, torch.bfloat16, torch.float32
    P = cfg.max_positions + POS_OFFSET
    yield "shared", (cfg.vocab_size, d), bf
    yield "final_logits_bias", (cfg.vocab_size,), f32
    for side, L in (("enc", cfg.enc_layers), ("dec", cfg.dec_layers)):
        yield f"{side}.pos", (P, d), bf
        yield f"{side}.ln_emb_g", (d,), f32
        yield f"{side}.ln_emb_b", (d,), f32
        for i in range(L):
            p = f"{side}.l{i}."
            yield p + "qkv_w", (3 * d, d), bf
            yield p + "qkv_b", (3 * d,), f32
            yield p + "o_w", (d, d), bf
            yield p + "o_b", (d,), f32
            yield p + "ln1_g", (d,), f32
            yield p + "ln1_b", (d,), f32
            if side == "dec":
                yield p + "cq_w", (d, d), bf
                yield p + "cq_b", (d,), f32
                yield p + "co_w", (d, d), bf
                yield p + "co_b", (d,), f32
                yield p + "lnc_g", (d,), f32
                yield p + "lnc_b", (d,), f32
            yield p + "f1_w", (f, d), bf
            yield p + "f1_b", (f,), f32
            yield p + "f2_w", (d, f), bf
            yield p + "f2_b", (d,), f32
            yield p + "ln2_g", (d,), f32
            yield p + "ln2_b", (d,), f32
    yield "dec.ckv_w", (cfg.dec_layers * 2 * d, d), bf  # every layer's cross K|V, one GEMM
    yield "dec.ckv_b", (cfg.dec_layers * 2 * d,), f32


def init_random(cfg: BartConfig, seed: int = 0, std: float = 0.02, device="cpu") -> ParamPack:
    """Seeded random init (HF BART scheme: N(0, init_std)-like weights, zero biases, LN = 1/0),
    built on ``device`` with the same bits everywhere (``params.rand_fill``)."""
    pack = ParamPack(param_specs(cfg), device=device)
    for name in pack.names():
        t = pack[name]
        base = name.split(".")[-1]
        if base.endswith("_g"):
            t.fill_(1.0)
        elif base.endswith("_b") or name == "final_logits_bias":
            pass  # zeros
        else:
            rand_fill(t, seed, name, std)
    return pack


def from_hf_state_dict(cfg: BartConfig, sd: Dict[str, torch.Tensor]) -> ParamPack:
    pack = ParamPack(param_specs(cfg))

    def put(name, t):
        pack[name].copy_(t.to(pack[name].dtype).view(pack[name].shape))

    put("shared", sd["model.shared.weight"])
    put("final_logits_bias", sd["final_logits_bias"].reshape(-1))
    ckv_w, ckv_b = [], []
    for side, hf, L in (("enc", "model.encoder", cfg.enc_layers), ("dec", "model.decoder", cfg.dec_layers)):
        put(f"{side}.pos", sd[f"{hf}.embed_positions.weight"])
        put(f"{side}.ln_emb_g", sd[f"{hf}.layernorm_embedding.weight"])
        put(f"{side}.ln_emb_b", sd[f"{hf}.layernorm_embedding.bias"])
        for i in range(L):
            b, p = f"{hf}.layers.{i}.", f"{side}.l{i}."
            a = b + "self_attn."
            put(p + "qkv_w", torch.cat([sd[a + f"{n}_proj.weight"] for n in "qkv"], 0))
            put(p + "qkv_b", torch.cat([sd[a + f"{n}_proj.bias"] for n in "qkv"], 0))
            put(p + "o_w", sd[a + "out_proj.weight"])
            put(p + "o_b", sd[a + "out_proj.bias"])
            put(p + "ln1_g", sd[b + "self_attn_layer_norm.weight"])
            put(p + "ln1_b", sd[b + "self_attn_layer_norm.bias"])
            if side == "dec":
                c = b + "encoder_attn."
                put(p + "cq_w", sd[c + "q_proj.weight"])
                put(p + "cq_b", sd[c + "q_proj.bias"])
                put(p + "co_w", sd[c + "out_proj.weight"])
                put(p + "co_b", sd[c + "out_proj.bias"])
                put(p + "lnc_g", sd[b + "encoder_attn_layer_norm.weight"])
                put(p + "lnc_b", sd[b + "encoder_attn_layer_norm.bias"])
                ckv_w += [sd[c + "k_proj.weight"], sd[c + "v_proj.weight"]]
                ckv_b += [sd[c + "k_proj.bias"], sd[c + "v_proj.bias"]]
            put(p + "f1_w", sd[b + "fc1.weight"])
            put(p + "f1_b", sd[b + "fc1.bias"])
            put(p + "f2_w", sd[b + "fc2.weight"])
            put(p + "f2_b", sd[b + "fc2.bias"])
            put(p + "ln2_g", sd[b + "final_layer_norm.weight"])
            put(p + "ln2_b", sd[b + "final_layer_norm.bias"])
    put("dec.ckv_w", torch.cat(ckv_w, 0))
    put("dec.ckv_b", torch.cat(ckv_b, 0))
    return pack


class BartModel:
    """Device-agnostic BART with the T5Model interface (encode / new_cache / step).

    On a ROCm device every op is a HIP kernel; on CPU with ``fp32=True`` each
    op's PyTorch reference runs (the oracle of the GPU tests and of the HF
    parity test).
    """

    family = "bart"

    def __init__(self, cfg: BartConfig, pack: ParamPack, fp32: bool = False):
        self.cfg, self.pack = cfg, pack
        self.p = pack.with_dtype(torch.float32) if fp32 else {n: pack[n] for n in pack.names()}
        self.device = pack.buffer.device
        dt = self.p["shared"].dtype
        self._type0 = torch.zeros((2, cfg.d_model), dtype=dt, device=self.device)
        # decode QKV GEMM writes K|V straight into the KV cache (no kv_append pass)
        self.kv_scatter = (self.device.type == "cuda" and not fp32
                           and os.getenv("ATPU_KV_SCATTER", "1") not in ("0", "false", "no"))
        # decoder steps: every post-LN LayerNorm but the last folded into the GEMMs around it
        # (ops.linear row_ln / res_ln): 35 fewer launches per step at 12 layers
        self.ln_fold = (self.device.type == "cuda" and not fp32
                        and os.getenv("ATPU_DEC_LN_FOLD", "1") not in ("0", "false", "no"))
        self._lfold: Optional[Dict[str, torch.Tensor]] = None
        # encoder: the post-LN LayerNorms folded into the GEMMs around them, as BERT's encoder
        # (BertClassifier.encode_folded): 24 fewer full passes over [B*S, d] per encode
        self.enc_ln_fold = (self.device.type == "cuda" and not fp32
                            and os.getenv("ATPU_ENC_LN_FOLD", "1") not in ("0", "false", "no"))
        self._efold: Optional[Dict[str, torch.Tensor]] = None

    def ln_folded(self) -> Dict[str, torch.Tensor]:
        """Decoder weights with each LayerNorm folded into its consumers (built once).

        ``LN(x) @ W.T + b = rstd*(x @ W'.T) - rstd*mu*colsum(W') + b'`` (W' = W*gamma,
        b' = b + W@beta) for the GEMMs that read LN(x); the GEMM that adds LN(x) as its
        residual normalises the raw rows itself and carries beta in its bias."""
        if self._lfold is None:
            p, f = self.p, {}
            for i in range(self.cfg.dec_layers):
                q, prev = f"dec.l{i}.", f"dec.l{i - 1}."
                for name, ln in (("qkv", prev + "ln2"), ("cq", q + "ln1"), ("f1", q + "lnc")):
                    if name == "qkv" and i == 0:
                        continue  # layer 0 reads the embedding LayerNorm's output (materialised)
                    f[q + name + "_w"], f[q + name + "_c"], f[q + name + "_b"] = ops.fold_ln_into_linear(
                        p[q + name + "_w"], p[q + name + "_b"], p[ln + "_g"], p[ln + "_b"])
                for name, ln in (("o", prev + "ln2"), ("co", q + "ln1"), ("f2", q + "lnc")):
                    if name == "o" and i == 0:
                        continue
                    f[q + name + "_b"] = (p[q + name + "_b"].float() + p[ln + "_b"].float()).contiguous()
            self._lfold = f
        return self._lfold

    def enc_folded(self) -> Dict[str, torch.Tensor]:
        """Encoder weights with each post-LN LayerNorm folded into its consumers (built once,
        then the device is synchronised: concurrent encodes on other streams read them).

        QKV of layer i >= 1 consumes LN2 of layer i-1 and FFN1 consumes LN1: gamma into the
        weight, beta into the bias, plus column sums (:func:`ops.fold_ln_into_linear`); the
        out-proj / FFN2 residual is that LayerNorm's output: its beta goes into their bias."""
        if self._efold is None:
            p, f = self.p, {}
            for i in range(self.cfg.enc_layers):
                q, prev = f"enc.l{i}.", f"enc.l{i - 1}."
                if i > 0:
                    g2, b2 = p[prev + "ln2_g"], p[prev + "ln2_b"]
                    f[q + "qkv_w"], f[q + "qkv_c"], f[q + "qkv_b"] = ops.fold_ln_into_linear(
                        p[q + "qkv_w"], p[q + "qkv_b"], g2, b2)
                    f[q + "o_b"] = (p[q + "o_b"].float() + b2.float()).contiguous()
                f[q + "f1_w"], f[q + "f1_c"], f[q + "f1_b"] = ops.fold_ln_into_linear(
                    p[q + "f1_w"], p[q + "f1_b"], p[q + "ln1_g"], p[q + "ln1_b"])
                f[q + "f2_b"] = (p[q + "f2_b"].float() + p[q + "ln1_b"].float()).contiguous()
            torch.cuda.synchronize(self.device)
            self._efold = f
        return self._efold

    def _enc_fold_ok(self, M: int) -> bool:
        d, ff = self.cfg.d_model, self.cfg.d_ff
        # not under batch invariance: the fold applies from M >= 2048 rows only, so a short batch
        # would take the LayerNorm-pass encoder and round differently
        return (self.enc_ln_fold and not ops.batch_invariant() and self.cfg.enc_layers >= 2
                and ops.fold_ok(M, 3 * d, d) and ops.fold_ok(M, ff, d)
                and ops.fold_ok(M, d, ff))

    def _encode_folded(self, ids: torch.Tensor, lens: torch.Tensor, ckv_out: Optional[torch.Tensor] = None):
        """:meth:`encode` with the LayerNorms folded (BERT's scheme, bert.py ``encode_folded``):
        the residual stream stays raw (pre-LN sums); out-proj / FFN2 emit per-row (sum, sumsq)
        partials of their output, ``ln_finalize`` turns them into (rstd, rstd*mu), which the
        next FFN1 / QKV apply to the folded weights' product and the next FFN2 / out-proj to
        their residual. Only the last LayerNorm runs (its output feeds the cross K|V)."""
        cfg, p, f = self.cfg, self.p, self.enc_folded()
        B, S = ids.shape
        d, H, M, eps = cfg.d_model, cfg.heads, B * S, cfg.eps
        h0 = ops.embed_layernorm(ids, p["shared"], p["enc.pos"][POS_OFFSET:], self._type0, p["enc.ln_emb_g"],
                                 p["enc.ln_emb_b"], eps)
        part = torch.empty((d // 256, M, 2), dtype=torch.float32, device=ids.device)  # raw rows' partials
        fin = torch.empty((M, 2), dtype=torch.float32, device=ids.device)             # (rstd, rstd*mu)
        g = h0
        for i in range(cfg.enc_layers):
            q, prev = f"enc.l{i}.", f"enc.l{i - 1}."
            if i == 0:
                qkv = ops.linear(h0, p[q + "qkv_w"], p[q + "qkv_b"])
            else:  # consumes LN2_{i-1}(g); fin = its statistics (also the out-proj residual's)
                qkv = ops.linear_ln(g, f[q + "qkv_w"], f[q + "qkv_b"], in_fin=fin, colsum=f[q + "qkv_c"])
            ctx = ops.attention_packed(qkv, lens, B, S, H)
            if i == 0:
                a = ops.linear_ln(ctx, p[q + "o_w"], p[q + "o_b"], residual=h0, part_out=part)
            else:
                a = ops.linear_ln(ctx, p[q + "o_w"], f[q + "o_b"], residual=g, res_fin=fin,
                                  res_gamma=p[prev + "ln2_g"], part_out=part)
            ops.ln_finalize(part, d, eps, out=fin)  # LN1 statistics of a
            ff = ops.linear_ln(a, f[q + "f1_w"], f[q + "f1_b"], act="gelu", in_fin=fin, colsum=f[q + "f1_c"])
            g = ops.linear_ln(ff, p[q + "f2_w"], f[q + "f2_b"], residual=a, res_fin=fin, res_gamma=p[q + "ln1_g"],
                              part_out=part)
            ops.ln_finalize(part, d, eps, out=fin)  # LN2 statistics of g
        last = f"enc.l{cfg.enc_layers - 1}."
        h = ops.layernorm(g, p[last + "ln2_g"], p[last + "ln2_b"], eps)
        return h, ops.linear(h, p["dec.ckv_w"], p["dec.ckv_b"], out=ckv_out)

    def prepare_decode(self, S: int, T: int) -> None:
        """Build the lazily folded decoder weights before concurrent decode streams fork."""
        if self.ln_fold:
            self.ln_folded()

    def wrap_source(self, toks):
        return [self.cfg.bos_id] + list(toks) + [self.cfg.eos_id]

    # ------------------------------------------------------------- encoder
    def encode(self, ids: torch.Tensor, lens: torch.Tensor, ckv_out: Optional[torch.Tensor] = None):
        """ids [B, S] int32, lens [B] -> (enc [B*S, d], cross K|V [B*S, L*2d]);
        ``ckv_out``: a [B*S, L*2d] buffer the cross K|V is written into (cached decode graphs)."""
        cfg, p = self.cfg, self.p
        B, S = ids.shape
        H = cfg.heads
        if ids.is_cuda and self._enc_fold_ok(B * S):
            return self._encode_folded(ids, lens, ckv_out)
        h = ops.embed_layernorm(ids, p["shared"], p["enc.pos"][POS_OFFSET:], self._type0, p["enc.ln_emb_g"],
                                p["enc.ln_emb_b"], cfg.eps)
        for i in range(cfg.enc_layers):
            q = f"enc.l{i}."
            qkv = ops.linear(h, p[q + "qkv_w"], p[q + "qkv_b"])
            ctx = ops.attention_packed(qkv, lens, B, S, H)
            h1 = ops.linear(ctx, p[q + "o_w"], p[q + "o_b"], residual=h)
            h1 = ops.layernorm(h1, p[q + "ln1_g"], p[q + "ln1_b"], cfg.eps)
            f = ops.linear(h1, p[q + "f1_w"], p[q + "f1_b"], act="gelu")
            h2 = ops.linear(f, p[q + "f2_w"], p[q + "f2_b"], residual=h1)
            h = ops.layernorm(h2, p[q + "ln2_g"], p[q + "ln2_b"], cfg.eps)
        return h, ops.linear(h, p["dec.ckv_w"], p["dec.ckv_b"], out=ckv_out)

    # ------------------------------------------------------------- decoder
    def new_cache(self, rows: int, T: int) -> torch.Tensor:
        """Self-attention K|V cache [L, rows*T, 2d]."""
        dt = self.p["dec.l0.qkv_w"].dtype
        return torch.zeros((self.cfg.dec_layers, rows * T, 2 * self.cfg.d_model), dtype=dt, device=self.device)

    def dec_embed(self) -> Optional["ops.DecEmbed"]:
        """The decoder input ``LN(shared[tok] + pos[step + 2])`` for ops.decode_advance to write
        (device bf16 model; None: the step embeds its tokens itself)."""
        p = self.p
        if not (p["shared"].is_cuda and p["shared"].dtype == torch.bfloat16 and self.cfg.d_model in (512, 768, 1024)):
            return None
        return ops.DecEmbed(p["shared"], p["dec.pos"], POS_OFFSET, p["dec.ln_emb_g"], p["dec.ln_emb_b"], self.cfg.eps)

    def step(self, tokens: torch.Tensor, step: torch.Tensor, cache: torch.Tensor, T: int, ckv: torch.Tensor,
             src_lens: torch.Tensor, S: int, group: int, hist: Optional[torch.Tensor] = None, logits: bool = True,
             x0: Optional[torch.Tensor] = None):
        """One decoder position for ``rows`` sequences -> fp32 logits [rows, V] (see T5Model.step)."""
        cfg, p = self.cfg, self.p
        d, H = cfg.d_model, cfg.heads
        scale = (d // H) ** -0.5
        # token + learned position (device-side step) + LayerNorm in one launch; x0: the input
        # ops.decode_advance already wrote (dec_embed)
        x = x0 if x0 is not None else ops.embed_pos_layernorm(tokens, p["shared"], p["dec.pos"], step, POS_OFFSET,
                                                              p["dec.ln_emb_g"], p["dec.ln_emb_b"], cfg.eps)
        if self.ln_fold:
            return self._step_folded(x, step, cache, T, ckv, src_lens, S, group, hist, logits)
        for i in range(cfg.dec_layers):
            q = f"dec.l{i}."
            c = cache[i]
            if self.kv_scatter:  # K|V written straight into the cache by the GEMM (no kv_append)
                qh = ops.linear(x, p[q + "qkv_w"], p[q + "qkv_b"], kv_cache=(c, T, step, d))
            else:
                qkv = ops.linear(x, p[q + "qkv_w"], p[q + "qkv_b"])
                ops.kv_append(qkv, d, 2 * d, c, T, step)
                qh = qkv[:, :d]
            ctx = ops.decode_attention(qh, c[:, :d], c[:, d:], H, T, 1, step=step, scale=scale, hist=hist)
            x = ops.layernorm(ops.linear(ctx, p[q + "o_w"], p[q + "o_b"], residual=x), p[q + "ln1_g"],
                              p[q + "ln1_b"], cfg.eps)
            cq = ops.linear(x, p[q + "cq_w"], p[q + "cq_b"])
            kv = ckv[:, i * 2 * d:(i + 1) * 2 * d]
            ctx = ops.decode_attention(cq, kv[:, :d], kv[:, d:], H, S, group, lens=src_lens, scale=scale)
            x = ops.layernorm(ops.linear(ctx, p[q + "co_w"], p[q + "co_b"], residual=x), p[q + "lnc_g"],
                              p[q + "lnc_b"], cfg.eps)
            f = ops.linear(x, p[q + "f1_w"], p[q + "f1_b"], act="gelu")
            x = ops.layernorm(ops.linear(f, p[q + "f2_w"], p[q + "f2_b"], residual=x), p[q + "ln2_g"],
                              p[q + "ln2_b"], cfg.eps)
        return ops.lm_head(x, p["shared"], p["final_logits_bias"], 0.0, logits)

    def _gemv_path(self, rows: int) -> bool:
        """The folded step's GEMMs all run on the <= 4-row GEMV (the library's own test, so
        ATPU_GEMV / ATPU_GEMM_TILE / shape / epilogue cannot disagree with the folding plan)."""
        from ..ops.linear import EPI_BIAS, EPI_GELU, EPI_KV_SCATTER, EPI_RES_LN, EPI_RESIDUAL, EPI_ROW_LN
        from .._native import native

        cfg, nat = self.cfg, native()
        d, kv = cfg.d_model, (EPI_KV_SCATTER if self.kv_scatter else 0)
        return (nat.gemv_selected(rows, 3 * d, EPI_ROW_LN | EPI_BIAS | kv)
                and nat.gemv_selected(rows, d, EPI_ROW_LN | EPI_BIAS)
                and nat.gemv_selected(rows, cfg.d_ff, EPI_ROW_LN | EPI_BIAS | EPI_GELU)
                and nat.gemv_selected(rows, d, EPI_BIAS | EPI_RESIDUAL | EPI_RES_LN))

    def _step_folded(self, x, step, cache, T, ckv, src_lens, S, group, hist, logits=True):
        """:meth:`step` with the decoder LayerNorms folded into the GEMMs (only the last one
        runs as a pass). The GEMM producing a pre-LN row writes its partial (sum, sumsq) per
        32-column slab; the GEMM reading LN(x) as input and the one adding LN(x) as its
        residual both normalise from those partials. On <= 4 rows (the decode GEMV) the GEMV
        reading LN(x) as input takes x's statistics from the rows it loads and hands them on
        to the residual consumer (``row_ln_out``), so the producers need no partials. Logits
        equal the unfolded step to bf16 rounding (tests/kernels/test_decode_gpu.py)."""
        cfg, p, f = self.cfg, self.p, self.ln_folded()
        d, H, eps, L = cfg.d_model, cfg.heads, cfg.eps, cfg.dec_layers
        scale = (d // H) ** -0.5
        # partials of: the layer input (last FFN2 out), the self-attention block out, the cross block out
        px, p1, p2 = torch.empty((3, d // 32, x.shape[0], 2), dtype=torch.float32, device=x.device).unbind(0)
        gemv = x.is_cuda and os.environ.get("ATPU_BART_SELF_STATS", "1") != "0" and self._gemv_path(x.shape[0])
        so = (lambda t: None) if gemv else (lambda t: t)  # producer partials: not on the GEMV path
        ro = (lambda t: t) if gemv else (lambda t: None)  # row_ln consumer hands x's statistics on
        inp = (lambda t: None) if gemv else (lambda t: t)  # the GEMV row_ln reads none
        for i in range(L):
            q, prev = f"dec.l{i}.", f"dec.l{i - 1}."
            c = cache[i]
            # layer 0: x = the embedding LayerNorm's output; later: raw pre-LN rows of the last FFN
            w, b, rl, rlo = ((p[q + "qkv_w"], p[q + "qkv_b"], None, None) if i == 0 else
                             (f[q + "qkv_w"], f[q + "qkv_b"], (eps, f[q + "qkv_c"], inp(px)), ro(px)))
            # each <= 4-row GEMV pulls the next one's weight into L2 (ops.linear prefetch; the
            # stats_out GEMVs have 32 weight rows per workgroup)
            rpb = 16 if gemv else 32
            nxt = f[f"dec.l{i + 1}.qkv_w"] if i + 1 < L else None
            if self.kv_scatter:
                qh = ops.linear(x, w, b, kv_cache=(c, T, step, d), row_ln=rl, row_ln_out=rlo,
                                prefetch=(p[q + "o_w"], rpb))
            else:
                qkv = ops.linear(x, w, b, row_ln=rl, row_ln_out=rlo, prefetch=(p[q + "o_w"], rpb))
                ops.kv_append(qkv, d, 2 * d, c, T, step)
                qh = qkv[:, :d]
            # the cross query projection's weight: prefetched by the o GEMV on the GEMV path
            ctx = ops.decode_attention(qh, c[:, :d], c[:, d:], H, T, 1, step=step, scale=scale, hist=hist)
            if i == 0:
                x1 = ops.linear(ctx, p[q + "o_w"], p[q + "o_b"], residual=x, stats_out=so(p1), prefetch=f[q + "cq_w"])
            else:
                x1 = ops.linear(ctx, p[q + "o_w"], f[q + "o_b"], residual=x, res_ln=(eps, px, p[prev + "ln2_g"]),
                                stats_out=so(p1), prefetch=f[q + "cq_w"])
            cq = ops.linear(x1, f[q + "cq_w"], f[q + "cq_b"], row_ln=(eps, f[q + "cq_c"], inp(p1)), row_ln_out=ro(p1),
                            prefetch=(p[q + "co_w"], rpb))
            kv = ckv[:, i * 2 * d:(i + 1) * 2 * d]
            ctx = ops.decode_attention(cq, kv[:, :d], kv[:, d:], H, S, group, lens=src_lens, scale=scale)
            x2 = ops.linear(ctx, p[q + "co_w"], f[q + "co_b"], residual=x1, res_ln=(eps, p1, p[q + "ln1_g"]),
                            stats_out=so(p2), prefetch=f[q + "f1_w"])
            h = ops.linear(x2, f[q + "f1_w"], f[q + "f1_b"], act="gelu", row_ln=(eps, f[q + "f1_c"], inp(p2)),
                           row_ln_out=ro(p2), prefetch=(p[q + "f2_w"], rpb))
            x = ops.linear(h, p[q + "f2_w"], f[q + "f2_b"], residual=x2, res_ln=(eps, p2, p[q + "lnc_g"]),
                           stats_out=so(px), prefetch=nxt)
        x = ops.layernorm(x, p[f"dec.l{L - 1}.ln2_g"], p[f"dec.l{L - 1}.ln2_b"], eps)
        return ops.lm_head(x, p["shared"], p["final_logits_bias"], 0.0, logits)
