"""ops_loader — resolve a list of op names to handlers at agent start-up.

Same API as the reference (``/root/reference/ops_loader.py:8-19``):
``load_ops(names) -> {name: handler}``, failing fast with ``ValueError`` for an
unknown or disabled op. :func:`load_ops_lenient` is what ``app.py`` uses: it
returns the loadable subset plus the per-op errors so the agent can start and
advertise only what it can actually run (fix for SURVEY.md §2.4.1).
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Iterable, List, Tuple

from ops import get_op

Handler = Callable[..., Any]


def load_ops(tasks: Iterable[str]) -> Dict[str, Handler]:
    return {name: get_op(name) for name in tasks}


def load_ops_lenient(tasks: Iterable[str]) -> Tuple[Dict[str, Handler], List[Tuple[str, str]]]:
    ok: Dict[str, Handler] = {}
    bad: List[Tuple[str, str]] = []
    for name in tasks:
        try:
            ok[name] = get_op(name)
        except Exception as exc:
            bad.append((name, str(exc)))
    return ok, bad
