"""``sat_verify`` — check a truth assignment against a CNF formula.

Mapped but missing in the reference (``/root/reference/ops/__init__.py:23``);
contract is new (sat_verify.CONTRACT.md; parity unpinned). Literals use the
DIMACS convention: variable ``v >= 1`` is ``v``, its negation ``-v``.
"""
from __future__ import annotations

from typing import Any, Dict, List

from . import register_op
from ._common import fail, is_int

MAX_CLAUSES = 1_000_000


def _assignment(raw: Any) -> Dict[int, bool]:
    if isinstance(raw, dict):
        return {int(k): bool(v) for k, v in raw.items()}
    if isinstance(raw, list):
        # list form: either booleans indexed from variable 1, or signed literals
        if all(isinstance(x, bool) for x in raw):
            return {i + 1: v for i, v in enumerate(raw)}
        if all(is_int(x) and x != 0 for x in raw):
            return {abs(x): x > 0 for x in raw}
    raise ValueError("payload.assignment must be {var: bool}, [bool...] or [signed literal...]")


@register_op("sat_verify")
def sat_verify(payload: Any) -> Dict[str, Any]:
    payload = payload or {}
    if not isinstance(payload, dict):
        return fail("payload must be a dict")
    cnf = payload.get("cnf")
    if not isinstance(cnf, list) or len(cnf) > MAX_CLAUSES:
        return fail("payload.cnf must be a list of clauses (lists of non-zero ints)")
    try:
        asg = _assignment(payload.get("assignment"))
    except (ValueError, TypeError) as exc:
        return fail(str(exc))
    unsat: List[int] = []
    unassigned = set()
    for ci, clause in enumerate(cnf):
        if not isinstance(clause, list) or not all(is_int(l) and l != 0 for l in clause):
            return fail(f"payload.cnf[{ci}] must be a list of non-zero integers")
        ok = False
        for lit in clause:
            val = asg.get(abs(lit))
            if val is None:
                unassigned.add(abs(lit))
                continue
            if val == (lit > 0):
                ok = True
                break
        if not ok:
            unsat.append(ci)
    return {"ok": True, "satisfied": not unsat, "clauses": len(cnf), "unsatisfied_clauses": unsat[:1000],
            "unsatisfied_count": len(unsat), "unassigned_vars": sorted(unassigned)[:1000]}
