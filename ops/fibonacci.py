"""``fibonacci`` — F(n) by fast doubling (O(log n) big-int multiplications).

The reference maps this op (``/root/reference/ops/__init__.py:21``) but ships no
module, so the contract is new (fibonacci.CONTRACT.md; parity unpinned).
"""
from __future__ import annotations

from typing import Any, Dict, Tuple

from . import register_op
from ._common import fail, is_int, js_int

MAX_N = 1_000_000


def fib_pair(n: int) -> Tuple[int, int]:
    """(F(n), F(n+1)) by fast doubling."""
    a, b = 0, 1
    for bit in bin(n)[2:]:
        c = a * (2 * b - a)
        d = a * a + b * b
        a, b = (d, c + d) if bit == "1" else (c, d)
    return a, b


@register_op("fibonacci")
def fibonacci(payload: Any) -> Dict[str, Any]:
    payload = payload or {}
    if not isinstance(payload, dict):
        return fail("payload must be a dict")
    n = payload.get("n")
    if not is_int(n) or n < 0:
        return fail("payload.n must be a non-negative integer")
    if n > MAX_N:
        return fail(f"payload.n must be <= {MAX_N}")
    count = payload.get("count", 1)
    if not is_int(count) or not 1 <= count <= 10_000:
        return fail("payload.count must be an integer in [1, 10000]")
    a, b = fib_pair(n)
    seq = [a]
    for _ in range(count - 1):
        a, b = b, a + b
        seq.append(a)
    out: Dict[str, Any] = {"ok": True, "n": n, "value": js_int(seq[0]), "digits": len(str(seq[0]))}
    if count > 1:
        out["sequence"] = [js_int(v) for v in seq]
    return out
