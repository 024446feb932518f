"""Fused masked attention (K4). Native kernel: ``csrc/kernels/attention.hip``.

* :func:`attention_packed` — BERT layout, ``qkv[B*S, 3*H*64]`` -> ``[B*S, H*64]``.
* :func:`attention` — strided q/k/v (T5 self/cross/causal attention) with an
  optional additive fp32 position bias ``[H, Sq, Skv]``.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .._native import native, ptr, launch_stream
from ._util import check, check_bf16_dev, row_stride, same_device

HEAD_DIM = 64


def dist_to_dense(bias_dist: torch.Tensor, Sq: int, Skv: int) -> torch.Tensor:
    """[H, Sq+Skv-1] bias by distance (entry k - q + Sq - 1) -> dense [H, Sq, Skv]."""
    idx = torch.arange(Skv, device=bias_dist.device).view(1, Skv) - torch.arange(Sq, device=bias_dist.device).view(Sq, 1)
    return bias_dist[:, idx + Sq - 1]


def attention_ref(q, k, v, lens, B, Sq, Skv, H, scale, bias=None, causal=False):
    """fp32 reference. q [B*Sq, >=H*D], k/v [B*Skv, >=H*D] (head h at cols h*D)."""
    D = HEAD_DIM
    qf = q[:, :H * D].float().view(B, Sq, H, D).transpose(1, 2)
    kf = k[:, :H * D].float().view(B, Skv, H, D).transpose(1, 2)
    vf = v[:, :H * D].float().view(B, Skv, H, D).transpose(1, 2)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if bias is not None:
        s = s + bias.float().unsqueeze(0)
    keys = torch.arange(Skv, device=q.device)
    dead = keys.view(1, 1, 1, Skv) >= lens.view(B, 1, 1, 1).to(q.device)
    if causal:
        dead = dead | (keys.view(1, 1, 1, Skv) > torch.arange(Sq, device=q.device).view(1, 1, Sq, 1))
    s = s.masked_fill(dead, float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    o = (p @ vf).transpose(1, 2).reshape(B * Sq, H * D)
    return o.to(q.dtype)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, lens: torch.Tensor, B: int, Sq: int, Skv: int,
              H: int, scale: Optional[float] = None, bias: Optional[torch.Tensor] = None, causal: bool = False,
              out: Optional[torch.Tensor] = None, bias_dist: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Masked multi-head attention (K4). ``bias``: dense fp32 [H, Sq, Skv]; ``bias_dist``:
    fp32 [H, Sq+Skv-1] indexed by key - query + Sq - 1 (T5 relative positions), which the
    kernel stages per head in LDS instead of streaming a dense S x S tensor."""
    scale = 1.0 / math.sqrt(HEAD_DIM) if scale is None else float(scale)
    check(bias is None or bias_dist is None, "attention: bias and bias_dist are exclusive")
    if bias_dist is not None:
        check(not causal, "attention: bias_dist is for non-causal (encoder) attention")
        check(bias_dist.dtype == torch.float32 and bias_dist.is_contiguous()
              and tuple(bias_dist.shape) == (H, Sq + Skv - 1), "bias_dist must be fp32 [H, Sq+Skv-1]")
        check(Sq + Skv - 1 <= 4096, "attention: bias_dist needs Sq + Skv - 1 <= 4096")
    if not q.is_cuda:
        if bias_dist is not None:
            bias = dist_to_dense(bias_dist.float(), Sq, Skv)
        o = attention_ref(q, k, v, lens, B, Sq, Skv, H, scale, bias, causal)
        if out is not None:
            out.copy_(o)
            return out
        return o
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        check_bf16_dev(t, n)
    check(q.shape[0] == B * Sq and k.shape[0] == B * Skv and v.shape[0] == B * Skv, "row counts must be B*S")
    check(q.shape[1] >= H * HEAD_DIM, "q narrower than H*64")
    check(lens.dtype == torch.int32 and lens.is_cuda and lens.numel() >= B, "lens must be int32 [B] on device")
    if bias is not None:
        check(bias.dtype == torch.float32 and bias.is_contiguous() and tuple(bias.shape) == (H, Sq, Skv),
              "bias must be fp32 [H, Sq, Skv]")
    if bias_dist is not None:
        same_device(q, bias_dist)
    if out is None:
        out = torch.empty((B * Sq, H * HEAD_DIM), dtype=torch.bfloat16, device=q.device)
    native().attention_strided(ptr(q), row_stride(q, "q"), ptr(k), row_stride(k, "k"), ptr(v), row_stride(v, "v"),
                               ptr(out), row_stride(out, "out"), ptr(lens), ptr(bias), B, Sq, Skv, H, HEAD_DIM,
                               scale, int(causal), launch_stream(q), ptr(bias_dist))
    return out


def attention_packed(qkv: torch.Tensor, lens: torch.Tensor, B: int, S: int, H: int,
                     out: Optional[torch.Tensor] = None, scale: Optional[float] = None) -> torch.Tensor:
    hd = H * HEAD_DIM
    check(qkv.dim() == 2 and qkv.shape[1] == 3 * hd, "qkv must be [B*S, 3*H*64]")
    return attention(qkv[:, :hd], qkv[:, hd:2 * hd], qkv[:, 2 * hd:], lens, B, S, S, H, scale=scale, out=out)
