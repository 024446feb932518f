"""Fused linear layer on the bf16 MFMA GEMM (K3/K5/K6).

``y = act(x @ w.T + bias) + residual`` with ``w`` in ``nn.Linear.weight``
layout ``[N, K]``. Native kernel: ``csrc/kernels/gemm_bf16.hip``. Skinny
problems (decode steps, M = beams x docs) run split-K: fp32 partials in a
caching-allocator workspace, summed in slice order by a reduce kernel that
applies the epilogue.
"""
from __future__ import annotations

import functools
from typing import Optional

import torch
import torch.nn.functional as F

from .._native import native, ptr, stream_handle
from ._util import check, check_bf16_dev, row_stride, same_device

EPI_BIAS, EPI_GELU, EPI_TANH, EPI_RESIDUAL, EPI_RELU, EPI_OUT_F32 = 1, 2, 4, 8, 16, 32
_ACTS = {None: 0, "none": 0, "gelu": EPI_GELU, "tanh": EPI_TANH, "relu": EPI_RELU}


def linear_ref(x, w, bias=None, act=None, residual=None, out_f32=False):
    y = x.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = F.gelu(y)
    elif act == "tanh":
        y = torch.tanh(y)
    elif act == "relu":
        y = torch.relu(y)
    if residual is not None:
        y = y + residual.float()
    return y if out_f32 else y.to(x.dtype)


@functools.lru_cache(maxsize=4096)
def _splits(M: int, N: int, K: int) -> int:
    return native().gemm_splitk_splits(M, N, K)


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: Optional[str] = None,
           residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           out_f32: bool = False) -> torch.Tensor:
    """``act(x @ w.T + bias) + residual``; ``out_f32`` returns fp32 (LM-head logits)."""
    check(act in _ACTS, f"unknown activation {act!r}")
    if not x.is_cuda:
        y = linear_ref(x, w, bias, act, residual, out_f32)
        if out is not None:
            out.copy_(y)
            return out
        return y
    check_bf16_dev(x, "x")
    check_bf16_dev(w, "w")
    same_device(x, w, bias, residual, out)
    M, K = x.shape
    N, K2 = w.shape
    check(K == K2, f"inner dims differ: x {tuple(x.shape)} w {tuple(w.shape)}")
    lda, ldb = row_stride(x, "x"), row_stride(w, "w")
    epi = _ACTS[act]
    if bias is not None:
        check(bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == N, "bias must be fp32 [N]")
        epi |= EPI_BIAS
    ldr = 0
    if residual is not None:
        check_bf16_dev(residual, "residual")
        check(tuple(residual.shape) == (M, N), "residual must be [M, N]")
        ldr = row_stride(residual, "residual")
        epi |= EPI_RESIDUAL
    if out_f32:
        epi |= EPI_OUT_F32
    odt = torch.float32 if out_f32 else torch.bfloat16
    if out is None:
        out = torch.empty((M, N), dtype=odt, device=x.device)
    check(tuple(out.shape) == (M, N) and out.dtype == odt, "out must be [M, N] of the output dtype")
    ldc = row_stride(out, "out")
    splits = _splits(M, N, K)
    ws = torch.empty(splits * M * N, dtype=torch.float32, device=x.device) if splits > 1 else None
    native().gemm(ptr(x), lda, ptr(w), ldb, ptr(out), ldc, ptr(bias), ptr(residual), ldr, M, N, K, epi,
                  stream_handle(), splits, ptr(ws))
    return out
