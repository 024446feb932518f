"""Row normalisation and embedding ops (K2, K6b, T5 RMSNorm).

Native kernels: ``csrc/kernels/norm_embed.hip`` (one wave per row, fp32 stats).
Row width must be a multiple of 256 (768 / 1024 for BERT, 768 for T5-base).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .._native import native, ptr, launch_stream
from ._util import check, check_bf16_dev


def _f32(t: torch.Tensor, n: int, name: str) -> None:
    check(t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n, f"{name} must be fp32 [{n}]")


def _check_out(out: torch.Tensor, shape, like: torch.Tensor) -> None:
    """A caller-provided output must be a contiguous bf16 tensor of the result's shape on the input's device."""
    check(tuple(out.shape) == tuple(shape), f"out must be {list(shape)}, got {list(out.shape)}")
    check(out.dtype == torch.bfloat16 and out.is_contiguous(), "out must be contiguous bf16")
    check(out.device == like.device, f"out is on {out.device}, inputs on {like.device}")


def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-12,
              residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    rows, N = x.shape
    if not x.is_cuda:
        y = x.float() + (residual.float() if residual is not None else 0.0)
        y = F.layer_norm(y, (N,), gamma.float(), beta.float(), eps).to(x.dtype)
        return out.copy_(y) if out is not None else y
    check_bf16_dev(x, "x")
    check(x.is_contiguous(), "x must be contiguous")
    _f32(gamma, N, "gamma")
    _f32(beta, N, "beta")
    if residual is not None:
        check_bf16_dev(residual, "residual")
        check(residual.is_contiguous() and residual.shape == x.shape, "residual must match x")
    if out is None:
        out = torch.empty_like(x)
    else:
        _check_out(out, x.shape, x)
    native().layernorm(ptr(x), ptr(residual), ptr(gamma), ptr(beta), ptr(out), rows, N, float(eps), launch_stream(x))
    return out


def rmsnorm(x: torch.Tensor, gamma: torch.Tensor, eps: float = 1e-6, out: Optional[torch.Tensor] = None):
    rows, N = x.shape
    if not x.is_cuda:
        xf = x.float()
        y = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()).to(x.dtype)
        return out.copy_(y) if out is not None else y
    check_bf16_dev(x, "x")
    check(x.is_contiguous(), "x must be contiguous")
    _f32(gamma, N, "gamma")
    if out is None:
        out = torch.empty_like(x)
    else:
        _check_out(out, x.shape, x)
    native().rmsnorm(ptr(x), ptr(gamma), ptr(out), rows, N, float(eps), launch_stream(x))
    return out


def embed_layernorm(ids: torch.Tensor, word: torch.Tensor, pos: torch.Tensor, type_: torch.Tensor,
                    gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-12,
                    type_ids: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``LN(word[ids] + pos[s] + type[type_ids])`` for ``ids[B, S]`` -> ``[B*S, N]``."""
    B, S = ids.shape
    V, N = word.shape
    if not ids.is_cuda:
        tt = type_ids if type_ids is not None else torch.zeros_like(ids)
        x = (word.float()[ids.long().clamp(0, V - 1)] + pos.float()[:S].unsqueeze(0)
             + type_.float()[tt.long().clamp(0, type_.shape[0] - 1)])
        y = F.layer_norm(x, (N,), gamma.float(), beta.float(), eps).to(word.dtype).view(B * S, N)
        return out.copy_(y) if out is not None else y
    check(ids.dtype == torch.int32 and ids.is_contiguous(), "ids must be contiguous int32")
    check(pos.shape[0] >= S, "sequence longer than the position table")
    for t, n in ((word, "word"), (pos, "pos"), (type_, "type")):
        check_bf16_dev(t, n)
    _f32(gamma, N, "gamma")
    _f32(beta, N, "beta")
    if type_ids is not None:
        check(type_ids.dtype == torch.int32 and type_ids.shape == ids.shape, "type_ids must be int32 [B,S]")
    check(tuple(pos.shape[1:]) == (N,) and tuple(type_.shape[1:]) == (N,) and type_.shape[0] > 0,
          "pos/type tables must be [*, N]")
    if out is None:
        out = torch.empty((B * S, N), dtype=torch.bfloat16, device=ids.device)
    else:
        _check_out(out, (B * S, N), word)
    native().embed_layernorm(ptr(ids), ptr(type_ids), ptr(word), ptr(pos), ptr(type_), ptr(gamma), ptr(beta),
                             ptr(out), B, S, N, V, type_.shape[0], float(eps), launch_stream(ids))
    return out


def embed_gather(ids: torch.Tensor, table: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    V, N = table.shape
    flat = ids.reshape(-1)
    if not ids.is_cuda:
        y = table[flat.long().clamp(0, V - 1)]
        return out.copy_(y) if out is not None else y
    check(ids.dtype == torch.int32 and ids.is_contiguous(), "ids must be contiguous int32")
    check_bf16_dev(table, "table")
    if out is None:
        out = torch.empty((flat.numel(), N), dtype=torch.bfloat16, device=ids.device)
    else:
        _check_out(out, (flat.numel(), N), table)
    native().embed_gather(ptr(flat), ptr(table), ptr(out), flat.numel(), N, V, launch_stream(table))
    return out


def embed_pos_layernorm(ids: torch.Tensor, table: torch.Tensor, pos: torch.Tensor, step: torch.Tensor, pos_off: int,
                        gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5,
                        out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``LN(table[ids[r]] + pos[step + pos_off])`` for every row r of ``ids`` -> ``[rows, N]``.

    The decoder input of a learned-position model (BART) at one device-side step: one launch,
    bit for bit ``layernorm(embed_gather(ids, table), residual=pos[step + pos_off])`` and the
    position index stays on the device (graph-capturable, no host sync)."""
    V, N = table.shape
    flat = ids.reshape(-1)
    rows = flat.numel()
    if not ids.is_cuda:
        pi = (step.reshape(-1)[:1].long() + pos_off).clamp(0, pos.shape[0] - 1)
        x = table[flat.long().clamp(0, V - 1)]
        y = layernorm(x, gamma, beta, eps, residual=pos.index_select(0, pi).expand(rows, N).contiguous())
        return out.copy_(y) if out is not None else y
    check(flat.dtype == torch.int32 and flat.is_contiguous(), "ids must be contiguous int32")
    check(step.dtype == torch.int32 and step.is_cuda and step.numel() >= 1, "step must be a device int32 tensor")
    check_bf16_dev(table, "table")
    check_bf16_dev(pos, "pos")
    check(pos.is_contiguous() and tuple(pos.shape[1:]) == (N,) and pos.shape[0] > 0, "pos must be [P, N]")
    _f32(gamma, N, "gamma")
    _f32(beta, N, "beta")
    if out is None:
        out = torch.empty((rows, N), dtype=torch.bfloat16, device=ids.device)
    else:
        _check_out(out, (rows, N), table)
    native().embed_pos_layernorm(ptr(flat), ptr(table), ptr(pos), ptr(step), int(pos_off), pos.shape[0], ptr(gamma),
                                 ptr(beta), ptr(out), rows, N, V, float(eps), launch_stream(table))
    return out
