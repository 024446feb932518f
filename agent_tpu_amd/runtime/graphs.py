"""hipGraph capture helper.

``torch.cuda.graph`` synchronizes the whole device and empties the caching
allocator on entry, every time. With several searches in flight on their own
streams (``runtime/summarize.generate_concurrent``) each lazy capture therefore
drained the siblings' queued steps. :func:`capture_graph` captures on a side
stream ordered after the caller's, in ``thread_local`` mode (other threads — the
CSV stager, the result poster — may keep using HIP), without either side effect.
"""
from __future__ import annotations

from typing import Any, Callable, Optional, Tuple

import torch


def capture_graph(fn: Callable[[], Any], pool: Optional[Tuple[int, int]] = None) -> Tuple["torch.cuda.CUDAGraph", Any]:
    """Capture ``fn()`` into a new CUDAGraph; returns ``(graph, fn's outputs)``.

    The work is recorded, not run (replay it to run it). Memory allocated during
    capture comes from the graph's private pool, or ``pool`` (share one between
    graphs that replay in order)."""
    caller = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    side.wait_stream(caller)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        if pool is not None:
            g.capture_begin(pool=pool, capture_error_mode="thread_local")
        else:
            g.capture_begin(capture_error_mode="thread_local")
        try:
            out = fn()
        finally:
            g.capture_end()
    caller.wait_stream(side)
    return g, out
