"""BERT QKV projection + self-attention in one kernel (K3 + K4 fused).

Native kernel: ``csrc/kernels/qkv_attn.hip`` (``qkv_attention``). The QKV GEMM runs on
256 x 192 tiles, one tile = one head's Q | K | V for two 128-token sequences, and the tile's
epilogue computes that head's attention for both sequences from LDS: the [M, 3*H*64] QKV
tensor is never written or read back (ref ``/root/reference/models/bert.py`` runs the
projection and attention as separate framework ops).

The attention runs in the tile epilogue on all 8 waves (``256h``). A wave-specialised
variant (4 MFMA waves on the main loop, 4 waves staging operands and running the previous
tile's attention) measured ~2 % slower and was removed (docs/PERF_NOTES.md, round 5).

The kernels want the QKV weight rows (and bias / colsum) in head order, ``[h][Q 64 | K 64 |
V 64]``; :func:`qkv_head_order` is that permutation of the usual ``[Q | K | V]`` layout.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .._native import native, ptr, launch_stream
from ._util import check, check_bf16_dev, row_stride, same_device
from .attention import HEAD_DIM, attention_ref
from .linear import EPI_BIAS, EPI_IN_NORM

SEQ = 128  # one tile = 2 sequences of exactly 128 tokens


def qkv_head_order(heads: int, device=None) -> torch.Tensor:
    """Index ``p`` with ``w_h = w[p]``: row ``h*192 + t*64 + d`` <- ``t*heads*64 + h*64 + d``."""
    hd = heads * HEAD_DIM
    h = torch.arange(heads).view(heads, 1, 1)
    t = torch.arange(3).view(1, 3, 1)
    d = torch.arange(HEAD_DIM).view(1, 1, HEAD_DIM)
    return (t * hd + h * HEAD_DIM + d).reshape(-1).to(device)


def qkv_attention_ok(M: int, N: int, K: int, S: int) -> bool:
    """Shapes the fused kernel takes: S == 128, whole 256-row tiles, K a multiple of 128."""
    return (S == SEQ and M % 256 == 0 and N % 192 == 0 and K % 128 == 0 and K >= 256
            and M * K * 2 < (1 << 32) and N * K * 2 < (1 << 32))


def qkv_attention(x: torch.Tensor, w_h: torch.Tensor, b_h: torch.Tensor, lens: torch.Tensor, heads: int, *,
                  in_fin: Optional[torch.Tensor] = None, colsum_h: Optional[torch.Tensor] = None,
                  out: Optional[torch.Tensor] = None, scale: Optional[float] = None) -> torch.Tensor:
    """Context ``[M, heads*64]`` of BERT self-attention over ``x [M, K]`` (M = B * 128 rows).

    ``w_h [3*heads*64, K]`` / ``b_h`` / ``colsum_h``: the QKV projection in head order
    (:func:`qkv_head_order`). ``in_fin [M, 2]`` + ``colsum_h``: ``x`` holds raw LayerNorm
    inputs and the weights are folded (:func:`ops.fold_ln_into_linear`), as ``linear_ln``.
    Keys ``>= lens[b]`` are masked."""
    scale = 1.0 / math.sqrt(HEAD_DIM) if scale is None else float(scale)
    M, K = x.shape
    N = w_h.shape[0]
    hd = heads * HEAD_DIM
    check(N == 3 * hd and w_h.shape[1] == K, f"qkv_attention: w_h must be [{3 * hd}, {K}]")
    check(M % SEQ == 0, "qkv_attention: rows must be B * 128")
    B = M // SEQ
    if not x.is_cuda:
        inv = torch.argsort(qkv_head_order(heads))
        y = x.float() @ w_h.float().t()
        if in_fin is not None:
            y = y * in_fin[:, :1] - in_fin[:, 1:] * colsum_h.float().unsqueeze(0)
        qkv = (y + b_h.float())[:, inv].to(x.dtype)
        o = attention_ref(qkv[:, :hd], qkv[:, hd:2 * hd], qkv[:, 2 * hd:], lens, B, SEQ, SEQ, heads, scale)
        return out.copy_(o) if out is not None else o
    check_bf16_dev(x, "x")
    check_bf16_dev(w_h, "w_h")
    same_device(x, w_h, b_h, lens, in_fin, colsum_h, out)
    check(qkv_attention_ok(M, N, K, SEQ), f"qkv_attention: unsupported shape M={M} N={N} K={K}")
    check(b_h.dtype == torch.float32 and b_h.is_contiguous() and b_h.numel() == N, "b_h must be fp32 [N]")
    check(lens.dtype == torch.int32 and lens.is_contiguous() and lens.numel() >= B, "lens must be int32 [B]")
    epi = EPI_BIAS
    if in_fin is not None:
        check(in_fin.dtype == torch.float32 and in_fin.is_contiguous() and tuple(in_fin.shape) == (M, 2),
              "in_fin must be contiguous fp32 [M, 2]")
        check(colsum_h is not None and colsum_h.dtype == torch.float32 and colsum_h.is_contiguous()
              and colsum_h.numel() == N, "colsum_h must be fp32 [N]")
        epi |= EPI_IN_NORM
    if out is None:
        out = torch.empty((M, hd), dtype=torch.bfloat16, device=x.device)
    check(out.dtype == torch.bfloat16 and tuple(out.shape) == (M, hd) and out.stride(1) == 1
          and out.stride(0) % 8 == 0 and out.data_ptr() % 16 == 0, "out must be bf16 [M, heads*64], 16-B rows")
    native().qkv_attention(ptr(x), row_stride(x, "x"), ptr(w_h), row_stride(w_h, "w_h"), ptr(out), out.stride(0),
                           ptr(b_h), M, N, K, epi, ptr(in_fin), ptr(colsum_h), ptr(lens), scale, launch_stream(x))
    return out
