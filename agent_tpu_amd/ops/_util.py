from __future__ import annotations

from typing import Optional

import torch


def check(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(f"agent_tpu_amd: {msg}")


def check_bf16_dev(t: torch.Tensor, name: str) -> None:
    check(t.is_cuda, f"{name} must be a device tensor")
    check(t.dtype == torch.bfloat16, f"{name} must be bfloat16 (got {t.dtype})")


def row_stride(t: torch.Tensor, name: str) -> int:
    """Leading dimension of a 2-D row-major view (inner dim contiguous)."""
    check(t.dim() == 2, f"{name} must be 2-D")
    check(t.stride(1) == 1, f"{name} inner dimension must be contiguous")
    return t.stride(0)


def same_device(*ts: Optional[torch.Tensor]) -> None:
    devs = {t.device for t in ts if t is not None}
    check(len(devs) <= 1, f"tensors on different devices: {devs}")
