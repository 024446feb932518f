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


class DeviceStages:
    """Device-side stage timing: hipEvent pairs recorded on the
    streams that run each stage, resolved after the caller's synchronize.

    ``timing_ms`` then carries ``device_<stage>_ms`` (sum of that stage's event
    pairs, GPU time) and ``device_span_ms`` (first start to last end on the
    device timeline). With one compute stream the compute stages add up to the
    span minus the gaps; with concurrent slots they overlap and their sum
    exceeds it (``device_overlap`` = sum / span)."""

    def __init__(self) -> None:
        self.pairs = []  # (stage, start, end)

    @staticmethod
    def event(stream=None):
        import torch

        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def add(self, stage: str, start, end) -> None:
        self.pairs.append((stage, start, end))

    def resolve(self, out: Dict[str, float]) -> Dict[str, float]:
        if not self.pairs:
            return out
        ref = self.pairs[0][1]
        lo, hi, busy = 0.0, 0.0, 0.0
        for stage, a, b in self.pairs:
            ms = a.elapsed_time(b)
            key = f"device_{stage}_ms"
            out[key] = round(out.get(key, 0.0) + ms, 3)
            lo = min(lo, ref.elapsed_time(a))
            hi = max(hi, ref.elapsed_time(b))
            busy += ms
        out["device_span_ms"] = round(hi - lo, 3)
        out["device_overlap"] = round(busy / (hi - lo), 3) if hi > lo else 1.0
        self.pairs = []
        return out
