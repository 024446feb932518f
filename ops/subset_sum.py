"""``subset_sum`` — find indices of a subset of integers summing to a target.

Mapped but missing in the reference (``/root/reference/ops/__init__.py:24``);
contract is new (subset_sum.CONTRACT.md; parity unpinned). Exact: a bitset DP
over reachable sums (Python big-int shifts) when the value range allows it,
otherwise meet-in-the-middle for up to 44 items.
"""
from __future__ import annotations

from bisect import bisect_left
from typing import Any, Dict, List, Optional

from . import register_op
from ._common import fail, is_int

MAX_ITEMS = 10_000
MAX_DP_SPAN = 1 << 24
MAX_MITM = 44


def _dp(values: List[int], target: int) -> Optional[List[int]]:
    # shift everything by the sum of negatives so the DP runs over [0, span]
    neg = sum(v for v in values if v < 0)
    span = sum(abs(v) for v in values)
    t = target - neg
    if t < 0 or t > span:
        return None
    masks = [1]  # reachable-sum bitsets after each prefix (offset by neg)
    reach = 1
    for v in values:
        reach = reach | (reach << abs(v))
        masks.append(reach)
    if not (reach >> t) & 1:
        return None
    # walk back: item i was taken iff sum-|v_i| was reachable before it
    picked: List[int] = []
    cur = t
    for i in range(len(values) - 1, -1, -1):
        a = abs(values[i])
        if (masks[i] >> cur) & 1:
            continue
        picked.append(i)
        cur -= a
    # a negative value v contributes 0 when NOT taken and -|v| when taken in the
    # real sum; in the shifted space it contributes |v| when NOT taken
    chosen = set(i for i in picked)
    return sorted(i for i in range(len(values)) if (values[i] >= 0) == (i in chosen))


def _mitm(values: List[int], target: int) -> Optional[List[int]]:
    h = len(values) // 2
    left, right = values[:h], values[h:]

    def sums(vs):
        out = [(0, 0)]
        for i, v in enumerate(vs):
            out += [(s + v, m | (1 << i)) for s, m in out]
        return out

    rs = sorted(sums(right))
    keys = [s for s, _ in rs]
    for s, m in sums(left):
        j = bisect_left(keys, target - s)
        if j < len(keys) and keys[j] == target - s:
            rm = rs[j][1]
            return [i for i in range(h) if m >> i & 1] + [h + i for i in range(len(right)) if rm >> i & 1]
    return None


@register_op("subset_sum")
def subset_sum(payload: Any) -> Dict[str, Any]:
    payload = payload or {}
    if not isinstance(payload, dict):
        return fail("payload must be a dict")
    values, target = payload.get("values"), payload.get("target")
    if not isinstance(values, list) or not all(is_int(v) for v in values) or len(values) > MAX_ITEMS:
        return fail(f"payload.values must be a list of at most {MAX_ITEMS} integers")
    if not is_int(target):
        return fail("payload.target must be an integer")
    if sum(abs(v) for v in values) <= MAX_DP_SPAN:
        idx, method = _dp(values, target), "bitset_dp"
    elif len(values) <= MAX_MITM:
        idx, method = _mitm(values, target), "meet_in_the_middle"
    else:
        return fail("instance too large: value span > 2**24 and more than 44 items")
    out: Dict[str, Any] = {"ok": True, "found": idx is not None, "method": method}
    if idx is not None:
        out["indices"] = idx
        out["subset"] = [values[i] for i in idx]
    return out
