"""Pre-encoded JSON values inside a result dict.

The classify result's ``rows`` (and the columnar ``index``/``score``) are encoded by
the native encoder (``_atpu.topk_json``) straight from the top-k arrays, so a
node-sized shard never becomes per-row Python dicts. :class:`RawJSON` carries those
bytes through the result dict; :func:`dumps` splices them into the HTTP body. For
in-process readers (tests, a local caller) it behaves like the list it encodes,
decoding lazily on first access.
"""
from __future__ import annotations

import json
from typing import Any, List


class RawJSON:
    __slots__ = ("data", "_value")

    def __init__(self, data: bytes):
        self.data = bytes(data)
        self._value = None

    @property
    def value(self) -> Any:
        if self._value is None:
            self._value = json.loads(self.data)
        return self._value

    def __len__(self) -> int:
        return len(self.value)

    def __getitem__(self, i):
        return self.value[i]

    def __iter__(self):
        return iter(self.value)

    def __eq__(self, other) -> bool:
        return self.value == (other.value if isinstance(other, RawJSON) else other)

    def __repr__(self) -> str:
        return f"RawJSON({len(self.data)} bytes)"


_MARK = "\x00ATPU_RAW\x00"


def dumps(obj: Any) -> bytes:
    """``json.dumps(obj, separators=(",", ":"), allow_nan=False)`` as UTF-8 bytes, with
    every :class:`RawJSON` value spliced in verbatim."""
    raws: List[bytes] = []

    def default(o):
        if isinstance(o, RawJSON):
            raws.append(o.data)
            return _MARK
        raise TypeError(f"Object of type {type(o).__name__} is not JSON serializable")

    text = json.dumps(obj, separators=(",", ":"), allow_nan=False, default=default)
    if not raws:
        return text.encode("utf-8")
    token = json.dumps(_MARK).encode("utf-8")  # the marker as json.dumps escapes it
    parts = text.encode("utf-8").split(token)
    if len(parts) != len(raws) + 1:
        raise ValueError("raw JSON marker collided with payload text")
    out = [parts[0]]
    for raw, tail in zip(raws, parts[1:]):
        out.append(raw)
        out.append(tail)
    return b"".join(out)


def plain(obj: Any) -> Any:
    """Deep copy with every :class:`RawJSON` decoded (for callers that need plain data)."""
    if isinstance(obj, RawJSON):
        return obj.value
    if isinstance(obj, dict):
        return {k: plain(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [plain(v) for v in obj]
    return obj
