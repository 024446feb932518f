"""``map_tokenize`` — fixed-size character chunking.

Parity with ``/root/reference/ops/map_tokenize.py:6-61``. The reference's
"tokens" are character chunks (not subwords); the subword/word ids that feed
BERT are produced on the GPU by ``map_classify`` (see map_classify.CONTRACT.md).
Errors are *returned* as ``{"ok": False, "error": ...}``, never raised.
"""
from __future__ import annotations

from typing import Any, Dict, List

from . import register_op

DEFAULT_CHUNK = 1024


def chunk_text(text: str, size: int) -> List[str]:
    """Split ``text`` into consecutive ``size``-character pieces."""
    return [text[pos:pos + size] for pos in range(0, len(text), size)] if text else []


def _bad(msg: str) -> Dict[str, Any]:
    return {"ok": False, "error": msg}


@register_op("map_tokenize")
def map_tokenize(payload: Any) -> Dict[str, Any]:
    payload = payload or {}
    size = payload.get("chunk_size", DEFAULT_CHUNK)
    # bool is an int subclass in Python; the reference accepts it (True == 1)
    if not isinstance(size, int) or size <= 0:
        return _bad("payload.chunk_size must be a positive integer")

    items = payload.get("items")
    if "items" in payload and items is not None:
        if not isinstance(items, list):
            return _bad("payload.items must be a list of strings")
        pieces: List[str] = []
        n_chars = 0
        for item in items:
            s = "" if item is None else str(item)
            n_chars += len(s)
            pieces += chunk_text(s, size)
        return {"ok": True, "tokens": pieces, "count": len(pieces),
                "total_chars": n_chars, "items_count": len(items)}

    text = payload.get("text") or payload.get("data", "")
    if not isinstance(text, str):
        return _bad("payload.text must be a string")
    pieces = chunk_text(text, size)
    return {"ok": True, "tokens": pieces, "count": len(pieces), "total_chars": len(text)}
