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


class DeviceMismatch(ValueError):
    pass


def check_launch_device(operand_dev: "torch.device", current_index: int) -> None:
    """Kernels take raw pointers and launch on the CURRENT device's stream, so
    operands on another GPU would be dereferenced by the wrong device (a memory
    access fault without peer access). Refuse it instead."""
    if operand_dev.type != "cuda":
        raise DeviceMismatch(f"kernel operand on {operand_dev}, expected a ROCm device tensor")
    idx = operand_dev.index if operand_dev.index is not None else current_index
    if idx != current_index:
        raise DeviceMismatch(f"kernel operands are on cuda:{idx} but the current device (launch stream) is "
                             f"cuda:{current_index}; wrap the call in torch.cuda.device({idx})")


def launch_stream(t: torch.Tensor) -> int:
    """The hipStream_t a kernel over ``t`` is launched on: the current stream of
    ``t``'s device, which must be the current device (:func:`check_launch_device`)."""
    cur = torch.cuda.current_device()
    check_launch_device(t.device, cur)
    return int(torch.cuda.current_stream(cur).cuda_stream)


def ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())
