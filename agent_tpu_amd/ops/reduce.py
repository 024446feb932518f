"""Streaming count/sum/min/max in fp64 (K12) for ``risk_accumulate``.

Native kernels: ``csrc/kernels/head_reduce.hip``. The multi-GPU variant (RCCL
all-reduce of the per-rank partials) is the ``risk_accumulate`` DP task in
:mod:`agent_tpu_amd.parallel.dp_ops` (:func:`~agent_tpu_amd.parallel.dp_ops.risk_task`).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Union

import torch

from .._native import native, ptr, launch_stream
from ._util import check


def reduce_stats_tensor(x: torch.Tensor) -> torch.Tensor:
    """Return fp64 ``[count, sum, min, max]`` on x's device."""
    check(x.dim() == 1 and x.is_contiguous(), "x must be a contiguous vector")
    if not x.is_cuda:
        xd = x.double()
        if xd.numel() == 0:
            return torch.tensor([0.0, 0.0, float("inf"), float("-inf")], dtype=torch.float64)
        return torch.stack([torch.tensor(float(xd.numel()), dtype=torch.float64), xd.sum(), xd.min(), xd.max()])
    check(x.dtype in (torch.float64, torch.float32), "x must be fp32 or fp64")
    nat = native()
    n = x.numel()
    blocks = nat.reduce_stats_blocks(n)
    partial = torch.empty(4 * blocks, dtype=torch.float64, device=x.device)
    out = torch.empty(4, dtype=torch.float64, device=x.device)
    s = launch_stream(x)
    if x.dtype == torch.float64:
        nat.reduce_stats_f64(ptr(x), n, ptr(partial), blocks, s)
    else:
        nat.reduce_stats_f32(ptr(x), n, ptr(partial), blocks, s)
    nat.reduce_stats_finalize(ptr(partial), blocks, ptr(out), s)
    return out


def stats_dict(v: Sequence[float]) -> Dict[str, Union[int, float, None]]:
    cnt = int(v[0])
    if cnt == 0:
        return {"count": 0, "sum": 0.0, "mean": 0.0, "min": None, "max": None}
    return {"count": cnt, "sum": float(v[1]), "mean": float(v[1]) / cnt, "min": float(v[2]), "max": float(v[3])}


def risk_stats(values: Union[List[float], torch.Tensor], device: str = "cuda") -> Dict[str, Union[int, float, None]]:
    x = values if isinstance(values, torch.Tensor) else torch.tensor(values, dtype=torch.float64)
    if device != "cpu" and torch.cuda.is_available():
        x = x.to(device, non_blocking=False)
    return stats_dict(reduce_stats_tensor(x.contiguous()).tolist())
