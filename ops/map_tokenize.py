"""``map_tokenize`` — fixed-size character chunking (the reference's "tokens").

Behaviour pinned to ``/root/reference/ops/map_tokenize.py:6-61`` by the
golden table in ``tests/contract/test_simple_ops.py``:
a "token" is a run of at most ``chunk_size`` characters, not a subword. The
word-piece ids that BERT consumes are produced on the GPU by ``map_classify``
(tokenizer kernel K1). Bad input is *returned* as ``{"ok": False, "error"}``.

Design: both payload shapes are normalised to one list of source strings
(``items`` entries, or the single ``text``/``data`` string), cut by a single
slicing pass; only the result keys differ between the two shapes.
"""
from __future__ import annotations

from itertools import chain
from typing import Any, Dict, Iterable, List, Optional, Tuple

from . import register_op

DEFAULT_CHUNK = 1024
_ERR_SIZE = "payload.chunk_size must be a positive integer"
_ERR_ITEMS = "payload.items must be a list of strings"
_ERR_TEXT = "payload.text must be a string"


def chunk_text(text: str, size: int) -> List[str]:
    """Consecutive ``size``-character slices of ``text`` (``[]`` for ``""``)."""
    return list(_slices(text, size))


def _slices(text: str, size: int) -> Iterable[str]:
    return (text[lo:lo + size] for lo in range(0, len(text), size))


def _sources(payload: Dict[str, Any]) -> Tuple[Optional[List[str]], bool, Optional[str]]:
    """-> (source strings, came from ``items``, error message)."""
    if payload.get("items") is not None:
        items = payload["items"]
        if not isinstance(items, list):
            return None, True, _ERR_ITEMS
        return ["" if it is None else str(it) for it in items], True, None
    # a falsy ``text`` ("" or None) falls through to ``data`` (reference behaviour)
    text = payload.get("text") or payload.get("data", "")
    if not isinstance(text, str):
        return None, False, _ERR_TEXT
    return [text], False, None


@register_op("map_tokenize")
def map_tokenize(payload: Any) -> Dict[str, Any]:
    payload = payload if payload is not None else {}
    size = payload.get("chunk_size", DEFAULT_CHUNK)
    # ``bool`` subclasses ``int``: True is accepted as size 1, like the reference
    if not (isinstance(size, int) and size > 0):
        return {"ok": False, "error": _ERR_SIZE}
    srcs, from_items, err = _sources(payload)
    if err is not None:
        return {"ok": False, "error": err}
    tokens = list(chain.from_iterable(_slices(s, size) for s in srcs))
    out: Dict[str, Any] = {"ok": True, "tokens": tokens, "count": len(tokens),
                           "total_chars": sum(map(len, srcs))}
    if from_items:
        out["items_count"] = len(srcs)
    return out
