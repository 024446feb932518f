"""Stage timing + roctx ranges.

``span(name, timings)`` measures a pipeline stage's wall time into
``timings[name]`` (milliseconds, accumulated) and, when ``MI355X_TRACE=1``,
brackets it with a roctx range so ``rocprofv3 --kernel-trace --marker-trace``
shows the host pipeline (CSV read, H2D, tokenize, encoder, head, collectives)
above the kernels. ``sync=True`` synchronizes the device first so GPU stages
are timed to completion (off by default: it would serialize the pipeline).
"""
from __future__ import annotations

import os
import time
from contextlib import contextmanager
from typing import Dict, Iterator, Optional

_ENABLED = os.getenv("MI355X_TRACE", "0").strip().lower() in ("1", "true")
_nat = None


def _native():
    global _nat
    if _nat is None:
        from .._native import native

        _nat = native()
    return _nat


def enabled() -> bool:
    return _ENABLED and bool(_native().trace_enabled())


@contextmanager
def span(name: str, timings: Optional[Dict[str, float]] = None, sync: bool = False) -> Iterator[None]:
    if _ENABLED:
        _native().trace_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if sync:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
        if timings is not None:
            timings[name] = timings.get(name, 0.0) + (time.perf_counter() - t0) * 1000.0
        if _ENABLED:
            _native().trace_pop()


def mark(name: str) -> None:
    if _ENABLED:
        _native().trace_mark(name)
