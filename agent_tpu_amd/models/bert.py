"""BERT sequence classifier on the hand-written gfx950 kernels.

Replaces the reference's opaque Edge-TPU ``interpreter.invoke()``
(``/root/reference/ops/map_classify_tpu.py:71-74``) with an explicit encoder:

    ids --K2 embed+LN--> h
    repeat L: qkv = h·Wqkvᵀ+b (K3) -> ctx = attn(qkv, lens) (K4)
              h1  = LN(ctx·Woᵀ+b+h)  (K5 + K6b)
              h   = LN(gelu(h1·W1ᵀ+b1)·W2ᵀ+b2+h1)  (K6, K5 + K6b)
    pooled = tanh(h[:,0]·Wpᵀ+bp) (GEMM, tanh epilogue, strided CLS rows)
    logits/top-k = head (K7)

Parameter names/layouts mirror HF ``BertForSequenceClassification`` (Linear
weights are ``[out, in]``, exactly the GEMM's ``Bt`` operand), so
:func:`from_hf_state_dict` is a rename plus the Q/K/V concat — used by the
parity test against transformers with identical random weights.
"""
from __future__ import annotations

import dataclasses
import math
import os
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from .. import ops
from .params import ParamPack, rand_fill


@dataclass(frozen=True)
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_positions: int = 512
    type_vocab: int = 2
    num_labels: int = 2
    eps: float = 1e-12

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    def param_count(self) -> int:
        H, I, L = self.hidden, self.intermediate, self.layers
        emb = (self.vocab_size + self.max_positions + self.type_vocab) * H + 2 * H
        layer = 4 * H * H + 4 * H + 2 * H * I + I + H + 4 * H
        head = H * H + H + self.num_labels * H + self.num_labels
        return emb + L * layer + head

    def flops_per_row_executed(self, seq_len: int, cls_only_last: bool = True) -> float:
        """FLOPs actually executed per row when the last layer runs on [CLS] only."""
        if not cls_only_last:
            return self.flops_per_row(seq_len)
        H, I, S = self.hidden, self.intermediate, seq_len
        full_layer = 2 * S * (4 * H * H + 2 * H * I) + 4 * S * S * H
        last = 2 * S * 2 * H * H + 2 * (2 * H * H + 2 * H * I) + 4 * S * H
        return self.flops_per_row(seq_len) - full_layer + last

    def flops_per_row(self, seq_len: int) -> float:
        """Forward FLOPs for one row of ``seq_len`` tokens (GEMMs + attention)."""
        H, I, L, S = self.hidden, self.intermediate, self.layers, seq_len
        gemm = 2 * S * (4 * H * H + 2 * H * I) * L
        attn = 4 * S * S * H * L
        head = 2 * (H * H + H * self.num_labels)
        return float(gemm + attn + head)


PRESETS: Dict[str, BertConfig] = {
    "bert-base": BertConfig(),
    "bert-large": BertConfig(hidden=1024, layers=24, heads=16, intermediate=4096),
    "bert-tiny": BertConfig(vocab_size=4096, hidden=256, layers=2, heads=4, intermediate=1024, max_positions=512),
}


def config_for(name: str, **overrides) -> BertConfig:
    if name not in PRESETS:
        raise ValueError(f"unknown BERT preset {name!r}; known: {sorted(PRESETS)}")
    return dataclasses.replace(PRESETS[name], **overrides)


def param_specs(cfg: BertConfig):
    H, I, C = cfg.hidden, cfg.intermediate, cfg.num_labels
    bf, f32 = torch.bfloat16, torch.float32
    yield "emb.word", (cfg.vocab_size, H), bf
    yield "emb.pos", (cfg.max_positions, H), bf
    yield "emb.type", (cfg.type_vocab, H), bf
    yield "emb.ln_g", (H,), f32
    yield "emb.ln_b", (H,), f32
    for i in range(cfg.layers):
        p = f"l{i}."
        yield p + "qkv_w", (3 * H, H), bf
        yield p + "qkv_b", (3 * H,), f32
        yield p + "o_w", (H, H), bf
        yield p + "o_b", (H,), f32
        yield p + "ln1_g", (H,), f32
        yield p + "ln1_b", (H,), f32
        yield p + "f1_w", (I, H), bf
        yield p + "f1_b", (I,), f32
        yield p + "f2_w", (H, I), bf
        yield p + "f2_b", (H,), f32
        yield p + "ln2_g", (H,), f32
        yield p + "ln2_b", (H,), f32
    yield "pool_w", (H, H), bf
    yield "pool_b", (H,), f32
    yield "cls_w", (C, H), bf
    yield "cls_b", (C,), f32


def init_random(cfg: BertConfig, seed: int = 0, std: float = 0.02, bias_std: float = 0.0,
                device="cpu") -> ParamPack:
    """Seeded random init, built where it will live: on a GPU by the ``rand_fill`` kernel
    (no host pass, no H2D copy), on the CPU by its native twin; the bits are the same on
    every device, host and rank (``params.rand_fill``).

    HF's BERT init scheme (N(0, 0.02)-like weights, LN γ=1/β=0, zero biases) unless
    ``bias_std`` > 0, which tests use to exercise the bias epilogues.
    """
    pack = ParamPack(param_specs(cfg), device=device)
    for name in pack.names():
        t = pack[name]
        if name.endswith("ln_g") or name.endswith("ln1_g") or name.endswith("ln2_g"):
            t.fill_(1.0)
        elif name.endswith("ln_b") or name.endswith("ln1_b") or name.endswith("ln2_b"):
            pass  # zeros
        elif name.endswith("_b"):
            if bias_std > 0:
                rand_fill(t, seed, name, bias_std)
        else:
            rand_fill(t, seed, name, std)
    return pack


def from_hf_state_dict(cfg: BertConfig, sd: Dict[str, torch.Tensor]) -> ParamPack:
    """Build a pack from a transformers ``BertForSequenceClassification`` state dict."""
    pack = ParamPack(param_specs(cfg))

    def put(name, t):
        pack[name].copy_(t.to(pack[name].dtype).view(pack[name].shape))

    put("emb.word", sd["bert.embeddings.word_embeddings.weight"])
    put("emb.pos", sd["bert.embeddings.position_embeddings.weight"])
    put("emb.type", sd["bert.embeddings.token_type_embeddings.weight"])
    put("emb.ln_g", sd["bert.embeddings.LayerNorm.weight"])
    put("emb.ln_b", sd["bert.embeddings.LayerNorm.bias"])
    for i in range(cfg.layers):
        b = f"bert.encoder.layer.{i}."
        a = b + "attention."
        put(f"l{i}.qkv_w", torch.cat([sd[a + f"self.{n}.weight"] for n in ("query", "key", "value")], 0))
        put(f"l{i}.qkv_b", torch.cat([sd[a + f"self.{n}.bias"] for n in ("query", "key", "value")], 0))
        put(f"l{i}.o_w", sd[a + "output.dense.weight"])
        put(f"l{i}.o_b", sd[a + "output.dense.bias"])
        put(f"l{i}.ln1_g", sd[a + "output.LayerNorm.weight"])
        put(f"l{i}.ln1_b", sd[a + "output.LayerNorm.bias"])
        put(f"l{i}.f1_w", sd[b + "intermediate.dense.weight"])
        put(f"l{i}.f1_b", sd[b + "intermediate.dense.bias"])
        put(f"l{i}.f2_w", sd[b + "output.dense.weight"])
        put(f"l{i}.f2_b", sd[b + "output.dense.bias"])
        put(f"l{i}.ln2_g", sd[b + "output.LayerNorm.weight"])
        put(f"l{i}.ln2_b", sd[b + "output.LayerNorm.bias"])
    put("pool_w", sd["bert.pooler.dense.weight"])
    put("pool_b", sd["bert.pooler.dense.bias"])
    put("cls_w", sd["classifier.weight"])
    put("cls_b", sd["classifier.bias"])
    return pack


class BertClassifier:
    """Encoder + pooler + classifier over a :class:`ParamPack`.

    ``params`` may live on a ROCm device (native kernels) or on the CPU (the
    PyTorch reference path of every op; pass ``fp32=True`` for an fp32 oracle).
    """

    def __init__(self, cfg: BertConfig, pack: ParamPack, fp32: bool = False, cls_only_last: Optional[bool] = None):
        self.cfg = cfg
        self.pack = pack
        self.p = pack.with_dtype(torch.float32) if fp32 else {n: pack[n] for n in pack.names()}
        self.device = pack.buffer.device
        # The classifier reads only the [CLS] row of the last layer (pooler on
        # h[:, 0]). So in that layer only K/V need every token; Q, attention
        # output, O-proj, LN and the FFN run on the B [CLS] rows. The logits are
        # those of the full computation; only dead rows are skipped.
        if cls_only_last is None:
            cls_only_last = os.getenv("ATPU_CLS_ONLY_LAST", "1") not in ("0", "false", "no")
        self.cls_only_last = bool(cls_only_last)
        # LayerNorm folding (GPU): no LayerNorm pass inside the encoder; see encode_folded
        self.ln_fold = (self.device.type == "cuda" and not fp32
                        and os.getenv("ATPU_LN_FOLD", "1") not in ("0", "false", "no"))
        self._folded: Optional[Dict[str, torch.Tensor]] = None
        # QKV projection + attention fused into one kernel (S = 128, LN-folded encoder):
        # ATPU_QKV_ATTN=0 runs the QKV GEMM and the packed attention kernel separately
        self.fused_qkv_attention = os.getenv("ATPU_QKV_ATTN", "1") not in ("0", "false", "no")

    # ------------------------------------------------------------ LN folding
    def folded(self) -> Dict[str, torch.Tensor]:
        """Weights with the preceding LayerNorm folded in (built once, on the device).

        QKV of layer i >= 1 consumes LN2 of layer i-1 and FFN1 of layer i consumes LN1
        of layer i: gamma goes into the weight, beta into the bias, plus the weight's
        column sums (:func:`ops.fold_ln_into_linear`). The out-proj / FFN2 residual is
        the same LayerNorm's output: its beta is added to their bias.
        """
        if self._folded is None:
            p, f = self.p, {}
            for i in range(self.cfg.layers):
                q = f"l{i}."
                if i > 0:
                    g2, b2 = p[f"l{i - 1}.ln2_g"], p[f"l{i - 1}.ln2_b"]
                    f[q + "qkv_w"], f[q + "qkv_c"], f[q + "qkv_b"] = ops.fold_ln_into_linear(
                        p[q + "qkv_w"], p[q + "qkv_b"], g2, b2)
                    f[q + "o_b"] = (p[q + "o_b"] + b2).contiguous()
                f[q + "f1_w"], f[q + "f1_c"], f[q + "f1_b"] = ops.fold_ln_into_linear(
                    p[q + "f1_w"], p[q + "f1_b"], p[q + "ln1_g"], p[q + "ln1_b"])
                f[q + "f2_b"] = (p[q + "f2_b"] + p[q + "ln1_b"]).contiguous()
                # head-ordered copies for the fused QKV + attention kernel ([h][Q|K|V] rows)
                perm = ops.qkv_head_order(self.cfg.heads, self.device)
                src = f if i > 0 else p
                f[q + "qkv_wh"] = src[q + "qkv_w"][perm].contiguous()
                f[q + "qkv_bh"] = src[q + "qkv_b"][perm].float().contiguous()
                if i > 0:
                    f[q + "qkv_ch"] = f[q + "qkv_c"][perm].contiguous()
            self._folded = f
        return self._folded

    def can_fold(self, B: int, S: int) -> bool:
        M, H, I = B * S, self.cfg.hidden, self.cfg.intermediate
        return (self.ln_fold and self.cfg.layers >= 2 and ops.fold_ok(M, 3 * H, H) and ops.fold_ok(M, I, H)
                and ops.fold_ok(M, H, I))

    def encode_folded(self, ids: torch.Tensor, lens: torch.Tensor, type_ids: Optional[torch.Tensor] = None,
                      cls_only_last: bool = False) -> torch.Tensor:
        """:meth:`encode` with every encoder LayerNorm folded into the GEMMs around it.

        The post-LN residual stream stays raw (pre-LN sums). The out-proj / FFN2
        epilogues emit per-row partial (sum, sumsq) of their output; a finalize pass
        turns them into (rstd, rstd*mu), which FFN1 / the next QKV apply to the
        folded weights' product and FFN2 / the next out-proj apply to their residual.
        Removes 2 LayerNorm passes per layer (each a full read + write of the hidden
        states); the logits match the unfolded encoder to bf16 rounding."""
        cfg, p, f = self.cfg, self.p, self.folded()
        B, S = ids.shape
        H, M, eps = cfg.hidden, B * S, cfg.eps
        dev = ids.device
        h0 = ops.embed_layernorm(ids, p["emb.word"], p["emb.pos"], p["emb.type"], p["emb.ln_g"], p["emb.ln_b"],
                                 eps, type_ids=type_ids)
        part = torch.empty((H // 256, M, 2), dtype=torch.float32, device=dev)  # raw rows' partials
        fin = torch.empty((M, 2), dtype=torch.float32, device=dev)             # (rstd, rstd*mu)
        last_full = cfg.layers - 1 if cls_only_last else cfg.layers
        fused = self.fused_qkv_attention and ops.qkv_attention_ok(M, 3 * H, H, S) and cfg.head_dim == 64
        g = h0
        for i in range(last_full):
            q = f"l{i}."
            if fused:
                # QKV projection + attention in one kernel: the [M, 3H] QKV tensor never exists
                ctx = ops.qkv_attention(g, f[q + "qkv_wh"], f[q + "qkv_bh"], lens, cfg.heads,
                                        in_fin=fin if i > 0 else None, colsum_h=f.get(q + "qkv_ch") if i > 0 else None)
            else:
                if i == 0:
                    qkv = ops.linear(h0, p[q + "qkv_w"], p[q + "qkv_b"])
                else:  # consumes LN2_{i-1}(g); fin = its statistics (also the out-proj residual's)
                    qkv = ops.linear_ln(g, f[q + "qkv_w"], f[q + "qkv_b"], in_fin=fin, colsum=f[q + "qkv_c"])
                ctx = ops.attention_packed(qkv, lens, B, S, cfg.heads)
            if i == 0:
                a = ops.linear_ln(ctx, p[q + "o_w"], p[q + "o_b"], residual=h0, part_out=part)
            else:
                a = ops.linear_ln(ctx, p[q + "o_w"], f[q + "o_b"], residual=g, res_fin=fin,
                                  res_gamma=p[f"l{i - 1}.ln2_g"], part_out=part)
            ops.ln_finalize(part, H, eps, out=fin)  # LN1 statistics of a
            ff = ops.linear_ln(a, f[q + "f1_w"], f[q + "f1_b"], act="gelu", in_fin=fin, colsum=f[q + "f1_c"])
            g = ops.linear_ln(ff, p[q + "f2_w"], f[q + "f2_b"], residual=a, res_fin=fin,
                              res_gamma=p[q + "ln1_g"], part_out=part)
            ops.ln_finalize(part, H, eps, out=fin)  # LN2 statistics of g
        ln2 = f"l{last_full - 1}."
        if not cls_only_last:
            return ops.layernorm(g, p[ln2 + "ln2_g"], p[ln2 + "ln2_b"], eps)
        # last layer on the [CLS] rows (see encode): K/V over every token from the raw g
        q = f"l{cfg.layers - 1}."
        kv = ops.linear_ln(g, f[q + "qkv_w"][H:], f[q + "qkv_b"][H:], in_fin=fin, colsum=f[q + "qkv_c"][H:])
        h_cls = ops.layernorm(g.view(B, S, H)[:, 0, :].contiguous(), p[ln2 + "ln2_g"], p[ln2 + "ln2_b"], eps)
        return self._cls_layer(h_cls, kv, lens, B, S)

    def _cls_layer(self, h_cls: torch.Tensor, kv: torch.Tensor, lens: torch.Tensor, B: int, S: int) -> torch.Tensor:
        """Last encoder layer on the [CLS] rows given their input and every token's K/V."""
        cfg, p, H = self.cfg, self.p, self.cfg.hidden
        q = f"l{cfg.layers - 1}."
        qc = ops.linear(h_cls, p[q + "qkv_w"][:H], p[q + "qkv_b"][:H])
        ctx = ops.decode_attention(qc, kv[:, :H], kv[:, H:], cfg.heads, S, 1, lens=lens,
                                   scale=1.0 / math.sqrt(cfg.head_dim))
        h1 = ops.linear(ctx, p[q + "o_w"], p[q + "o_b"], residual=h_cls.contiguous())
        h1 = ops.layernorm(h1, p[q + "ln1_g"], p[q + "ln1_b"], cfg.eps)
        f = ops.linear(h1, p[q + "f1_w"], p[q + "f1_b"], act="gelu")
        h2 = ops.linear(f, p[q + "f2_w"], p[q + "f2_b"], residual=h1)
        return ops.layernorm(h2, p[q + "ln2_g"], p[q + "ln2_b"], cfg.eps)

    def encode(self, ids: torch.Tensor, lens: torch.Tensor, type_ids: Optional[torch.Tensor] = None,
               cls_only_last: bool = False) -> torch.Tensor:
        """Hidden states ``[B*S, H]``, or ``[B, H]`` [CLS] states with ``cls_only_last``."""
        cfg, p = self.cfg, self.p
        B, S = ids.shape
        if ids.is_cuda and self.can_fold(B, S):
            return self.encode_folded(ids, lens, type_ids, cls_only_last)
        H = cfg.hidden
        h = ops.embed_layernorm(ids, p["emb.word"], p["emb.pos"], p["emb.type"], p["emb.ln_g"], p["emb.ln_b"],
                                cfg.eps, type_ids=type_ids)
        last_full = cfg.layers - 1 if cls_only_last else cfg.layers
        for i in range(last_full):
            q = f"l{i}."
            qkv = ops.linear(h, p[q + "qkv_w"], p[q + "qkv_b"])
            ctx = ops.attention_packed(qkv, lens, B, S, cfg.heads)
            h1 = ops.linear(ctx, p[q + "o_w"], p[q + "o_b"], residual=h)
            h1 = ops.layernorm(h1, p[q + "ln1_g"], p[q + "ln1_b"], cfg.eps)
            f = ops.linear(h1, p[q + "f1_w"], p[q + "f1_b"], act="gelu")
            h2 = ops.linear(f, p[q + "f2_w"], p[q + "f2_b"], residual=h1)
            h = ops.layernorm(h2, p[q + "ln2_g"], p[q + "ln2_b"], cfg.eps)
        if not cls_only_last:
            return h
        # last layer on the [CLS] rows: K/V GEMM over every token (rows H..3H of
        # the fused weight), Q GEMM over the B [CLS] rows, single-query attention
        q = f"l{cfg.layers - 1}."
        kv = ops.linear(h, p[q + "qkv_w"][H:], p[q + "qkv_b"][H:])
        h_cls = h.view(B, S, H)[:, 0, :]  # strided view: row stride S*H
        return self._cls_layer(h_cls, kv, lens, B, S)

    def pooled(self, h: torch.Tensor, B: int, S: int) -> torch.Tensor:
        cls_rows = h if h.shape[0] == B else h.view(B, S, self.cfg.hidden)[:, 0, :]  # strided: row stride S*H
        return ops.linear(cls_rows, self.p["pool_w"], self.p["pool_b"], act="tanh")

    def encoder(self, ids: torch.Tensor, lens: torch.Tensor,
                type_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The encoder stage of :meth:`forward` ([CLS] states when the last layer is pruned)."""
        return self.encode(ids, lens, type_ids, cls_only_last=self.cls_only_last and ids.shape[1] > 1)

    def head(self, h: torch.Tensor, B: int, S: int, k: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Pooler + classifier + softmax/top-k (K7) over encoder states ``h``."""
        pooled = self.pooled(h, B, S)
        return ops.classify_head_topk(pooled, self.p["cls_w"], self.p["cls_b"], k)

    def forward(self, ids: torch.Tensor, lens: torch.Tensor, k: int = 5,
                type_ids: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Returns ``(logits[B,C] fp32, topk_idx[B,k] int32, topk_prob[B,k] fp32)``."""
        B, S = ids.shape
        return self.head(self.encoder(ids, lens, type_ids), B, S, k)
