"""Small helpers shared by the CPU ops (payload validation in the reference's
``{"ok": False, "error": ...}`` style, see /root/reference/ops/map_tokenize.py:26)."""
from __future__ import annotations

from typing import Any, Dict

JS_SAFE = 2 ** 53


def fail(msg: str) -> Dict[str, Any]:
    return {"ok": False, "error": msg}


def is_int(x: Any) -> bool:
    return isinstance(x, int) and not isinstance(x, bool)


def js_int(v: int):
    """Integers beyond 2**53 lose precision in JSON consumers: send them as strings."""
    return v if -JS_SAFE < v < JS_SAFE else str(v)
