"""GPU tokenizer (K1): packed UTF-8 rows -> ``ids[B, S]``, ``lens[B]``.

Spec and pure-Python twin: :mod:`agent_tpu_amd.tokenizer`.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from .._native import native, ptr, launch_stream
from .. import tokenizer as _tok
from ._util import check


def tokenize(text: torch.Tensor, offsets: torch.Tensor, seq_len: int, vocab: int,
             max_row_bytes: int = _tok.DEFAULT_MAX_ROW_BYTES, ids: Optional[torch.Tensor] = None,
             lens: Optional[torch.Tensor] = None, rows: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    B = offsets.numel() - 1 if rows is None else rows
    if not text.is_cuda:
        t = np.ascontiguousarray(text.numpy(), dtype=np.uint8)
        o = np.ascontiguousarray(offsets.numpy()[:B + 1], dtype=np.int32)
        i, l = native().tokenize_host(t, o, seq_len, vocab, max_row_bytes)
        ids_t, lens_t = torch.from_numpy(i), torch.from_numpy(l)
        if ids is not None:
            ids[:B].copy_(ids_t)
            lens[:B].copy_(lens_t)
            return ids, lens
        return ids_t, lens_t
    check(text.dtype == torch.uint8 and offsets.dtype == torch.int32, "text uint8 / offsets int32")
    check(offsets.is_cuda and offsets.numel() >= B + 1, "offsets must be device int32 [B+1]")
    if ids is None:
        ids = torch.empty((B, seq_len), dtype=torch.int32, device=text.device)
        lens = torch.empty((B,), dtype=torch.int32, device=text.device)
    check(ids.shape[1] == seq_len and ids.shape[0] >= B and lens.numel() >= B, "ids/lens too small")
    native().tokenize(ptr(text), ptr(offsets), ptr(ids), ptr(lens), B, seq_len, vocab, max_row_bytes,
                      launch_stream(text), int(text.numel()))
    return ids, lens
