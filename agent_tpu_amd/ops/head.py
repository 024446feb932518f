"""Classifier head + softmax + top-k (K7). Native: ``csrc/kernels/head_reduce.hip``.

Top-k order: descending probability, ties to the lower class index (the
reference's ``_topk`` in ``/root/reference/ops/map_classify_tpu.py:15-19``
sorts by descending score; its tie order is unspecified).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._native import native, ptr, launch_stream
from ._util import check, check_bf16_dev, row_stride


def classify_head_topk_ref(pooled, Wc, bc, k):
    logits = pooled.float() @ Wc.float().t() + (bc.float() if bc is not None else 0.0)
    probs = torch.softmax(logits, dim=-1)
    # stable sort on -prob keeps lower index first among ties
    order = torch.sort(-probs, dim=-1, stable=True).indices[:, :k]
    return logits, order.to(torch.int32), torch.gather(probs, 1, order)


def classify_head_topk(pooled: torch.Tensor, Wc: torch.Tensor, bc: Optional[torch.Tensor], k: int,
                       logits: Optional[torch.Tensor] = None, idx: Optional[torch.Tensor] = None,
                       score: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    B, N = pooled.shape
    C = Wc.shape[0]
    k = max(1, min(int(k), C))
    if not pooled.is_cuda:
        return classify_head_topk_ref(pooled, Wc, bc, k)
    check_bf16_dev(pooled, "pooled")
    check_bf16_dev(Wc, "Wc")
    check(Wc.is_contiguous() and Wc.shape[1] == N, "Wc must be contiguous [C, N]")
    if bc is not None:
        check(bc.dtype == torch.float32 and bc.numel() == C, "bc must be fp32 [C]")
    dev = pooled.device
    logits = torch.empty((B, C), dtype=torch.float32, device=dev) if logits is None else logits
    idx = torch.empty((B, k), dtype=torch.int32, device=dev) if idx is None else idx
    score = torch.empty((B, k), dtype=torch.float32, device=dev) if score is None else score
    native().head_topk(ptr(pooled), row_stride(pooled, "pooled"), ptr(Wc), ptr(bc), ptr(logits), ptr(idx), ptr(score),
                       B, N, C, k, launch_stream(pooled))
    return logits, idx, score
