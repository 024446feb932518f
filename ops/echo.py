"""``echo`` — plumbing op: hands the payload straight back.

Parity with ``/root/reference/ops/echo.py:7-24``: ``None`` echoes ``{}``; a
non-dict payload is echoed with ``note: payload_was_not_dict``.
"""
from __future__ import annotations

from typing import Any, Dict

from . import register_op


@register_op("echo")
def echo(payload: Any) -> Dict[str, Any]:
    if payload is None:
        return {"ok": True, "echo": {}}
    out: Dict[str, Any] = {"ok": True, "echo": payload}
    if not isinstance(payload, dict):
        out["note"] = "payload_was_not_dict"
    return out
