"""T5 encoder-decoder on the gfx950 kernels (map_summarize, BASELINE config 4).

Replaces the reference's CPU ``BartForConditionalGeneration.generate``
(``/root/reference/ops/map_summarize.py:52-59``) with an explicit HIP path:

  encoder  : gather (K8) -> L x [RMSNorm, fused QKV GEMM, attention with the
             T5 bidirectional relative-position bias (K4 bias path), O-proj +
             residual (GEMM epilogue), RMSNorm, FFN ReLU (epilogue), FFN2 +
             residual] -> RMSNorm -> ONE GEMM producing every decoder layer's
             cross-attention K/V ([B*S, L*2d]).
  decoder  : per generated token, L x [RMSNorm, QKV GEMM, KV-cache append,
             single-query attention over the cache with the causal distance
             bias (K9), O-proj + residual, RMSNorm, cross Q GEMM, single-query
             cross attention over the encoder K/V (beams share their item's
             rows), O-proj + residual, RMSNorm, FFN] -> RMSNorm -> LM-head GEMM
             with fp32 logits -> fused log-softmax/top-k (K10).

Parameter names follow HF ``T5ForConditionalGeneration`` (Linear weights are
``[out, in]``) so :func:`from_hf_state_dict` is a rename + concat; T5 uses no
Linear biases, unscaled attention and RMSNorm (eps 1e-6). The tied LM head is
stored pre-scaled by ``d_model**-0.5`` (what HF applies at run time).
"""
from __future__ import annotations

import dataclasses
import math
import os
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from .. import ops
from .params import ParamPack, rand_fill


@dataclass(frozen=True)
class T5Config:
    vocab_size: int = 32128
    d_model: int = 768
    d_kv: int = 64
    d_ff: int = 3072
    heads: int = 12
    enc_layers: int = 12
    dec_layers: int = 12
    buckets: int = 32
    max_distance: int = 128
    eps: float = 1e-6
    pad_id: int = 0
    eos_id: int = 1
    decoder_start_id: int = 0
    tie_embeddings: bool = True

    def param_count(self) -> int:
        d, f = self.d_model, self.d_ff
        enc = self.enc_layers * (4 * d * d + 2 * d * f + 2 * d)
        dec = self.dec_layers * (8 * d * d + 2 * d * f + 3 * d)
        return self.vocab_size * d + enc + dec + 2 * d + 2 * self.buckets * self.heads


PRESETS: Dict[str, T5Config] = {
    "t5-base": T5Config(),
    "t5-small": T5Config(d_model=512, d_ff=2048, heads=8, enc_layers=6, dec_layers=6),
    "t5-tiny": T5Config(vocab_size=4096, d_model=256, d_ff=1024, heads=4, enc_layers=2, dec_layers=2),
}


def config_for(name: str, **overrides) -> T5Config:
    if name not in PRESETS:
        raise ValueError(f"unknown T5 preset {name!r}; known: {sorted(PRESETS)}")
    return dataclasses.replace(PRESETS[name], **overrides)


def param_specs(cfg: T5Config):
    d, f, bf, f32 = cfg.d_model, cfg.d_ff, torch.bfloat16, torch.float32
    yield "shared", (cfg.vocab_size, d), bf
    yield "enc.rel", (cfg.buckets, cfg.heads), f32
    for i in range(cfg.enc_layers):
        p = f"enc.l{i}."
        yield p + "ln1", (d,), f32
        yield p + "qkv", (3 * d, d), bf
        yield p + "o", (d, d), bf
        yield p + "ln2", (d,), f32
        yield p + "wi", (f, d), bf
        yield p + "wo", (d, f), bf
    yield "enc.ln_f", (d,), f32
    yield "dec.rel", (cfg.buckets, cfg.heads), f32
    for i in range(cfg.dec_layers):
        p = f"dec.l{i}."
        yield p + "ln1", (d,), f32
        yield p + "qkv", (3 * d, d), bf
        yield p + "o", (d, d), bf
        yield p + "ln2", (d,), f32
        yield p + "cq", (d, d), bf
        yield p + "co", (d, d), bf
        yield p + "ln3", (d,), f32
        yield p + "wi", (f, d), bf
        yield p + "wo", (d, f), bf
    yield "dec.ckv", (cfg.dec_layers * 2 * d, d), bf  # every layer's cross K|V, one GEMM
    yield "dec.ln_f", (d,), f32
    yield "lm", (cfg.vocab_size, d), bf


def init_random(cfg: T5Config, seed: int = 0, device="cpu") -> ParamPack:
    """Seeded random init (HF T5 scheme: factor 1.0 normal-like with fan-in scaling), built on
    ``device`` with the same bits everywhere (``params.rand_fill``)."""
    pack = ParamPack(param_specs(cfg), device=device)
    d, f = cfg.d_model, cfg.d_ff
    for name in pack.names():
        t = pack[name]
        base = name.split(".")[-1]
        if base.startswith("ln"):
            t.fill_(1.0)
        elif base == "rel":
            rand_fill(t, seed, name, d ** -0.5)
        elif name == "shared":
            rand_fill(t, seed, name, 1.0)
        elif base in ("wo",):
            rand_fill(t, seed, name, f ** -0.5)
        elif base == "qkv":
            # T5 folds the 1/sqrt(d_kv) attention scale into the q rows (the first d rows)
            rand_fill(t, seed, name, d ** -0.5 * cfg.d_kv ** -0.5, n0=d * t.shape[1], std1=d ** -0.5)
        elif base == "cq":
            rand_fill(t, seed, name, d ** -0.5 * cfg.d_kv ** -0.5)
        else:
            rand_fill(t, seed, name, d ** -0.5)
    if cfg.tie_embeddings:
        pack["lm"].copy_((pack["shared"].float() * d ** -0.5).to(torch.bfloat16))
    return pack


def from_hf_state_dict(cfg: T5Config, sd: Dict[str, torch.Tensor]) -> ParamPack:
    pack = ParamPack(param_specs(cfg))
    d = cfg.d_model

    def put(name, t):
        pack[name].copy_(t.to(pack[name].dtype).view(pack[name].shape))

    put("shared", sd["shared.weight"])
    put("enc.rel", sd["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"])
    for i in range(cfg.enc_layers):
        b = f"encoder.block.{i}.layer."
        put(f"enc.l{i}.ln1", sd[b + "0.layer_norm.weight"])
        put(f"enc.l{i}.qkv", torch.cat([sd[b + f"0.SelfAttention.{n}.weight"] for n in "qkv"], 0))
        put(f"enc.l{i}.o", sd[b + "0.SelfAttention.o.weight"])
        put(f"enc.l{i}.ln2", sd[b + "1.layer_norm.weight"])
        put(f"enc.l{i}.wi", sd[b + "1.DenseReluDense.wi.weight"])
        put(f"enc.l{i}.wo", sd[b + "1.DenseReluDense.wo.weight"])
    put("enc.ln_f", sd["encoder.final_layer_norm.weight"])
    put("dec.rel", sd["decoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"])
    ckv = []
    for i in range(cfg.dec_layers):
        b = f"decoder.block.{i}.layer."
        put(f"dec.l{i}.ln1", sd[b + "0.layer_norm.weight"])
        put(f"dec.l{i}.qkv", torch.cat([sd[b + f"0.SelfAttention.{n}.weight"] for n in "qkv"], 0))
        put(f"dec.l{i}.o", sd[b + "0.SelfAttention.o.weight"])
        put(f"dec.l{i}.ln2", sd[b + "1.layer_norm.weight"])
        put(f"dec.l{i}.cq", sd[b + "1.EncDecAttention.q.weight"])
        put(f"dec.l{i}.co", sd[b + "1.EncDecAttention.o.weight"])
        ckv += [sd[b + "1.EncDecAttention.k.weight"], sd[b + "1.EncDecAttention.v.weight"]]
        put(f"dec.l{i}.ln3", sd[b + "2.layer_norm.weight"])
        put(f"dec.l{i}.wi", sd[b + "2.DenseReluDense.wi.weight"])
        put(f"dec.l{i}.wo", sd[b + "2.DenseReluDense.wo.weight"])
    put("dec.ckv", torch.cat(ckv, 0))
    put("dec.ln_f", sd["decoder.final_layer_norm.weight"])
    lm = sd.get("lm_head.weight", sd["shared.weight"])
    put("lm", lm.float() * (d ** -0.5 if cfg.tie_embeddings else 1.0))
    return pack


def relative_bucket(rel: torch.Tensor, bidirectional: bool, buckets: int, max_distance: int) -> torch.Tensor:
    """T5 relative-position bucketing (same function as HF ``_relative_position_bucket``)."""
    out = torch.zeros_like(rel)
    if bidirectional:
        buckets //= 2
        out += (rel > 0).to(rel.dtype) * buckets
        rel = rel.abs()
    else:
        rel = -torch.clamp(rel, max=0)
    exact = buckets // 2
    small = rel < exact
    large = exact + (torch.log(rel.float().clamp(min=1) / exact) / math.log(max_distance / exact)
                     * (buckets - exact)).to(rel.dtype)
    large = torch.clamp(large, max=buckets - 1)
    return out + torch.where(small, rel, large)


class T5Model:
    """Device-agnostic T5: ``pack`` on a ROCm device runs the HIP kernels; on CPU
    (with ``fp32=True``) every op's PyTorch reference, used as the oracle."""

    family = "t5"

    def __init__(self, cfg: T5Config, pack: ParamPack, fp32: bool = False):
        self.cfg, self.pack = cfg, pack
        self.p = pack.with_dtype(torch.float32) if fp32 else {n: pack[n] for n in pack.names()}
        self.device = pack.buffer.device
        self._enc_bias: Dict[int, torch.Tensor] = {}
        self._dec_bias: Optional[torch.Tensor] = None
        # decoder steps: every RMSNorm folded into the GEMM that consumes it (gamma in the
        # weight, the row statistics summed in the GEMM's K loop; ops.linear rms_eps)
        self.rms_fold = (self.device.type == "cuda" and not fp32
                         and os.getenv("ATPU_RMS_FOLD", "1") not in ("0", "false", "no"))
        self._rfold: Optional[Dict[str, torch.Tensor]] = None
        self.kv_scatter = (self.device.type == "cuda" and not fp32
                           and os.getenv("ATPU_KV_SCATTER", "1") not in ("0", "false", "no"))

    def rms_folded(self) -> Dict[str, torch.Tensor]:
        """Decoder weights with the preceding RMSNorm's gamma folded in (built once)."""
        if self._rfold is None:
            p, f = self.p, {}
            for i in range(self.cfg.dec_layers):
                q = f"dec.l{i}."
                f[q + "qkv"] = ops.fold_rms_into_linear(p[q + "qkv"], p[q + "ln1"])
                f[q + "cq"] = ops.fold_rms_into_linear(p[q + "cq"], p[q + "ln2"])
                f[q + "wi"] = ops.fold_rms_into_linear(p[q + "wi"], p[q + "ln3"])
            f["lm"] = ops.fold_rms_into_linear(p["lm"], p["dec.ln_f"])
            self._rfold = f
        return self._rfold

    def wrap_source(self, toks):
        return list(toks) + [self.cfg.eos_id]

    def prepare_decode(self, S: int, T: int) -> None:
        """Build the lazily cached tensors a search of source length S / length T reads, on
        the caller's stream (concurrent searches on other streams then only read them)."""
        self.enc_bias_dist(S)
        self.dec_bias(T)
        if self.rms_fold:
            self.rms_folded()

    # ------------------------------------------------------------- biases
    def enc_bias_dist(self, S: int) -> torch.Tensor:
        """Encoder relative-position bias by distance: [H, 2S-1], entry k - q + S - 1
        (the attention kernel stages one head's row in LDS; no dense [H, S, S])."""
        key = -S
        if key not in self._enc_bias:
            rel_pos = torch.arange(-(S - 1), S)
            b = relative_bucket(rel_pos, True, self.cfg.buckets, self.cfg.max_distance)
            rel = self.p["enc.rel"].float().cpu()  # [buckets, H]
            self._enc_bias[key] = rel[b].t().contiguous().to(self.device)  # [H, 2S-1]
        return self._enc_bias[key]

    def dec_bias(self, T: int) -> torch.Tensor:
        if self._dec_bias is None or self._dec_bias.shape[1] < T:
            dist = torch.arange(T)
            b = relative_bucket(-dist, False, self.cfg.buckets, self.cfg.max_distance)
            rel = self.p["dec.rel"].float().cpu()
            self._dec_bias = rel[b].t().contiguous().to(self.device)  # [H, T] by distance q-k
        return self._dec_bias

    # ------------------------------------------------------------- encoder
    def encode(self, ids: torch.Tensor, lens: torch.Tensor, ckv_out: Optional[torch.Tensor] = None):
        """ids [B, S] int32 (S % 4 == 0), lens [B] -> (enc [B*S, d], cross K|V [B*S, L*2d]);
        ``ckv_out``: a [B*S, L*2d] buffer the cross K|V is written into (cached decode graphs)."""
        cfg, p = self.cfg, self.p
        B, S = ids.shape
        d, H = cfg.d_model, cfg.heads
        bias = self.enc_bias_dist(S)
        h = ops.embed_gather(ids, p["shared"])
        if h.dtype != p["enc.l0.qkv"].dtype:
            h = h.to(p["enc.l0.qkv"].dtype)
        for i in range(cfg.enc_layers):
            q = f"enc.l{i}."
            x = ops.rmsnorm(h, p[q + "ln1"], cfg.eps)
            qkv = ops.linear(x, p[q + "qkv"])
            ctx = ops.attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], lens, B, S, S, H, scale=1.0,
                                bias_dist=bias)
            h = ops.linear(ctx, p[q + "o"], residual=h)
            x = ops.rmsnorm(h, p[q + "ln2"], cfg.eps)
            f = ops.linear(x, p[q + "wi"], act="relu")
            h = ops.linear(f, p[q + "wo"], residual=h)
        enc = ops.rmsnorm(h, p["enc.ln_f"], cfg.eps)
        return enc, ops.linear(enc, p["dec.ckv"], out=ckv_out)

    # ------------------------------------------------------------- decoder
    def new_cache(self, rows: int, T: int) -> torch.Tensor:
        """Self-attention K|V cache [L, rows*T, 2d]."""
        dt = self.p["dec.l0.qkv"].dtype
        return torch.zeros((self.cfg.dec_layers, rows * T, 2 * self.cfg.d_model), dtype=dt, device=self.device)

    def dec_embed(self) -> Optional["ops.DecEmbed"]:
        """The decoder input (``shared[tok]``) for ops.decode_advance to write, on the device
        bf16 model (None: the step embeds its tokens itself)."""
        t = self.p["shared"]
        ok = t.is_cuda and t.dtype == torch.bfloat16 and self.cfg.d_model in (512, 768, 1024)
        return ops.DecEmbed(t) if ok else None

    def step(self, tokens: torch.Tensor, step: torch.Tensor, cache: torch.Tensor, T: int, ckv: torch.Tensor,
             src_lens: torch.Tensor, S: int, group: int, hist: Optional[torch.Tensor] = None, logits: bool = True,
             x0: Optional[torch.Tensor] = None):
        """One decoder position for ``rows`` sequences -> fp32 logits [rows, V]
        (``logits=False``: the :class:`ops.LmHead` input for the fused LM head + top-k).

        ``step`` is a 1-element int32 device tensor (position of ``tokens``);
        cache rows of sequence r are r*T .. r*T+T-1; encoder rows of batch item
        r // group are (r//group)*S ... ``hist`` (int32 [rows, T]) are beam
        backpointers: position j < step of row r was computed by row hist[r, j].
        Every argument is a device tensor, so the step is hipGraph-capturable.
        """
        cfg, p = self.cfg, self.p
        d, H = cfg.d_model, cfg.heads
        dbias = self.dec_bias(T)
        # x0: the input ops.decode_advance already embedded (dec_embed)
        x = x0 if x0 is not None else ops.embed_gather(tokens, p["shared"])
        if x.dtype != p["dec.l0.qkv"].dtype:
            x = x.to(p["dec.l0.qkv"].dtype)
        if self.rms_fold:
            return self._step_folded(x, step, cache, T, ckv, src_lens, S, group, hist, dbias, logits)
        for i in range(cfg.dec_layers):
            q = f"dec.l{i}."
            c = cache[i]
            y = ops.rmsnorm(x, p[q + "ln1"], cfg.eps)
            qkv = ops.linear(y, p[q + "qkv"])
            ops.kv_append(qkv, d, 2 * d, c, T, step)
            ctx = ops.decode_attention(qkv[:, :d], c[:, :d], c[:, d:], H, T, 1, step=step, bias_dist=dbias, hist=hist)
            x = ops.linear(ctx, p[q + "o"], residual=x)
            y = ops.rmsnorm(x, p[q + "ln2"], cfg.eps)
            cq = ops.linear(y, p[q + "cq"])
            kv = ckv[:, i * 2 * d:(i + 1) * 2 * d]
            ctx = ops.decode_attention(cq, kv[:, :d], kv[:, d:], H, S, group, lens=src_lens)
            x = ops.linear(ctx, p[q + "co"], residual=x)
            y = ops.rmsnorm(x, p[q + "ln3"], cfg.eps)
            f = ops.linear(y, p[q + "wi"], act="relu")
            x = ops.linear(f, p[q + "wo"], residual=x)
        y = ops.rmsnorm(x, p["dec.ln_f"], cfg.eps)
        return ops.lm_head(y, p["lm"], None, 0.0, logits)

    def _step_folded(self, x, step, cache, T, ckv, src_lens, S, group, hist, dbias, logits=True):
        """:meth:`step` with each RMSNorm folded into its consumer GEMM (37 fewer launches
        per step, no normalised copy of x); logits equal the unfolded step to bf16 rounding."""
        cfg, p, f = self.cfg, self.p, self.rms_folded()
        d, H, eps = cfg.d_model, cfg.heads, cfg.eps
        # each <= 4-row GEMV pulls the next one's weight into L2 (ops.linear prefetch)
        L = cfg.dec_layers
        nxt_qkv = [f[f"dec.l{i + 1}.qkv"] if i + 1 < L else None for i in range(L)]
        for i in range(L):
            q = f"dec.l{i}."
            c = cache[i]
            if self.kv_scatter:  # K|V written straight into the cache by the GEMM (no kv_append)
                qh = ops.linear(x, f[q + "qkv"], rms_eps=eps, kv_cache=(c, T, step, d), prefetch=p[q + "o"])
            else:
                qkv = ops.linear(x, f[q + "qkv"], rms_eps=eps, prefetch=p[q + "o"])
                ops.kv_append(qkv, d, 2 * d, c, T, step)
                qh = qkv[:, :d]
            ctx = ops.decode_attention(qh, c[:, :d], c[:, d:], H, T, 1, step=step, bias_dist=dbias, hist=hist)
            x = ops.linear(ctx, p[q + "o"], residual=x, prefetch=f[q + "cq"])
            cq = ops.linear(x, f[q + "cq"], rms_eps=eps, prefetch=p[q + "co"])
            kv = ckv[:, i * 2 * d:(i + 1) * 2 * d]
            ctx = ops.decode_attention(cq, kv[:, :d], kv[:, d:], H, S, group, lens=src_lens)
            x = ops.linear(ctx, p[q + "co"], residual=x, prefetch=f[q + "wi"])
            h = ops.linear(x, f[q + "wi"], act="relu", rms_eps=eps, prefetch=p[q + "wo"])
            x = ops.linear(h, p[q + "wo"], residual=x, prefetch=nxt_qkv[i])
        return ops.lm_head(x, f["lm"], None, eps, logits)
