"""Loader for the in-tree native extension ``agent_tpu_amd/_atpu*.so``.

``torch`` is imported first on purpose: the extension links
``libamdhip64.so.7`` and must bind to the HIP runtime torch already loaded
(same SONAME), so device pointers and streams are shared with PyTorch.

On a machine with a GPU a missing/broken extension is an error (never a
silent eager fallback); ``ATPU_REQUIRE_NATIVE=1`` forces that everywhere.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
from typing import Any, Optional

import torch  # noqa: F401  (must precede the extension import)

_mod: Optional[Any] = None
_err: Optional[BaseException] = None


class NativeUnavailable(RuntimeError):
    pass


def _try_build() -> None:
    if os.environ.get("ATPU_NO_AUTOBUILD", "0") == "1":
        return
    from .csrc import build as _b

    _b.build()


def native() -> Any:
    """Return the ``_atpu`` module, building it in-tree if it is missing."""
    global _mod, _err
    if _mod is not None:
        return _mod
    alt = os.environ.get("ATPU_NATIVE_PATH")
    if alt:  # development A/B: load another build of the extension (same module name)
        spec = importlib.util.spec_from_file_location("agent_tpu_amd._atpu", alt)
        _mod = importlib.util.module_from_spec(spec)
        sys.modules["agent_tpu_amd._atpu"] = _mod
        spec.loader.exec_module(_mod)
        return _mod
    try:
        _mod = importlib.import_module("agent_tpu_amd._atpu")
        return _mod
    except ImportError as exc:
        _err = exc
    try:
        _try_build()
        _mod = importlib.import_module("agent_tpu_amd._atpu")
        return _mod
    except Exception as exc:  # pragma: no cover - surfaced to caller
        _err = exc
        raise NativeUnavailable(f"agent_tpu_amd native extension unavailable: {exc}") from exc


def available() -> bool:
    try:
        native()
        return True
    except NativeUnavailable:
        return False


def stream_handle(stream: Optional["torch.cuda.Stream"] = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())
