"""Op registry for the MI355X job agent.

Behavioural parity with the reference registry (``/root/reference/ops/__init__.py``):

* ``register_op(name)`` decorator fills :data:`OPS_REGISTRY` at module import
  (ref ``ops/__init__.py:35-39``).
* ``TASKS`` env gating, re-read on every call: unset/blank/``*``/``all`` -> every
  default-enabled op, ``none`` -> nothing, otherwise an exact (case-sensitive)
  name set; the keywords themselves are case-insensitive (ref ``:42-71``).
* ``get_op(name)`` checks, in order: enabled -> known -> import module ->
  registered, raising ``ValueError`` with the reference's four messages
  (ref ``:87-108``).

Deliberate fixes:

* :data:`OP_TO_MODULE` only names modules that exist (§2.4.4); the four missing
  reference modules (fibonacci, prime_factor, sat_verify, subset_sum) are now
  real CPU ops.
* ``csv_shard`` and ``read_csv_shard`` both resolve (§2.4.5).
* ``map_classify`` (GPU BERT path) is registered under its own name and under
  the reference's ``map_classify_tpu`` name.
* Side-effecting ERP triggers are registered but OPT-IN: ``all``/unset does not
  enable them, only an explicit name in ``TASKS`` does (§2.4.6).
* A module whose import failed is not retried on every call; its error is
  recorded once (the reference appends a duplicate on every call).
"""
from __future__ import annotations

import importlib
import os
import threading
from typing import Any, Callable, Dict, FrozenSet, List, Optional, Set, Tuple

OpFn = Callable[..., Any]

OPS_REGISTRY: Dict[str, OpFn] = {}
#: op name -> handler over a LIST of payloads (same-op jobs of one lease, run as
#: one device batch); returns one ``("ok", result)`` / ``("err", exception)`` per payload
BATCH_REGISTRY: Dict[str, OpFn] = {}
OPS_LOAD_ERRORS: List[Tuple[str, str]] = []  # (module, "Type: message")

#: op name -> module file under ``ops/`` (every entry exists in this tree)
OP_TO_MODULE: Dict[str, str] = {
    # plumbing / CPU ops
    "echo": "echo",
    "map_tokenize": "map_tokenize",
    "csv_shard": "csv_shard",
    "read_csv_shard": "csv_shard",
    "risk_accumulate": "risk_accumulate",
    "fibonacci": "fibonacci",
    "prime_factor": "prime_factor",
    "sat_verify": "sat_verify",
    "subset_sum": "subset_sum",
    # MI355X accelerator ops
    "map_classify": "map_classify",
    "map_classify_tpu": "map_classify",
    "map_summarize": "map_summarize",
    # outbound side effects (opt-in only)
    "trigger_oracle": "trigger_oracle",
    "trigger_sap": "trigger_sap",
}

#: ops that ``TASKS=all`` / unset do NOT enable; they must be named explicitly
OPT_IN_OPS: FrozenSet[str] = frozenset({"trigger_oracle", "trigger_sap"})

_imported: Set[str] = set()
_failed: Dict[str, str] = {}
_lock = threading.Lock()


def register_op(name: str) -> Callable[[OpFn], OpFn]:
    """Decorator: ``@register_op("echo")`` makes ``fn`` resolvable by name."""

    def _wrap(fn: OpFn) -> OpFn:
        OPS_REGISTRY[name] = fn
        return fn

    return _wrap


def register_batch_op(name: str) -> Callable[[OpFn], OpFn]:
    """Decorator: ``fn(payloads) -> [("ok", result) | ("err", exc), ...]`` runs several
    jobs of op ``name`` as one batch. Every entry must equal what the single-job
    handler would return (or raise) for that payload; only the throughput differs."""

    def _wrap(fn: OpFn) -> OpFn:
        BATCH_REGISTRY[name] = fn
        return fn

    return _wrap


def get_batch_op(name: str) -> Optional[OpFn]:
    """The batch handler of an op already resolved by :func:`get_op` (or None)."""
    return BATCH_REGISTRY.get(name)


#: op name -> factory of a continuous (in-flight) executor: ``factory()`` returns an object
#: with ``submit(tag, payload)``, ``pump() -> [(tag, ("ok", result) | ("err", exc, trace))]``
#: and ``busy() -> bool``; jobs join a running device batch at its next step boundary
STREAM_REGISTRY: Dict[str, Callable[[], Any]] = {}


def register_stream_op(name: str) -> Callable[[Callable[[], Any]], Callable[[], Any]]:
    """Decorator: the in-flight executor factory of op ``name`` (app.py ``INFLIGHT_DEPTH``).
    As for batch handlers, every result must equal the single-job handler's."""

    def _wrap(fn):
        STREAM_REGISTRY[name] = fn
        return fn

    return _wrap


def get_stream_op(name: str) -> Optional[Callable[[], Any]]:
    return STREAM_REGISTRY.get(name)


def _enabled_set() -> Optional[Set[str]]:
    """Parse ``TASKS``. ``None`` means "all default ops"; a set is exact names."""
    names = [tok.strip() for tok in os.getenv("TASKS", "").split(",")]
    names = [n for n in names if n]
    if not names:
        return None
    keywords = {n.lower() for n in names}
    if keywords & {"*", "all"}:
        # keep explicitly-named opt-in ops on top of "all"
        return None if not (set(names) & OPT_IN_OPS) else {"*all*", *names}
    if "none" in keywords:
        return set()
    return set(names)


def _is_enabled(name: str) -> bool:
    enabled = _enabled_set()
    if enabled is None:
        return name not in OPT_IN_OPS
    if "*all*" in enabled:
        return name not in OPT_IN_OPS or name in enabled
    return name in enabled


def list_ops() -> List[str]:
    """Sorted names of known ops that the current ``TASKS`` enables."""
    return sorted(n for n in OP_TO_MODULE if _is_enabled(n))


def _import_module(module: str) -> None:
    with _lock:
        if module in _imported or module in _failed:
            return
        try:
            importlib.import_module(f"{__name__}.{module}")
        except Exception as exc:  # record once, keep the agent alive
            msg = f"{type(exc).__name__}: {exc}"
            _failed[module] = msg
            OPS_LOAD_ERRORS.append((module, msg))
            print(f"[ops] ERROR: failed to import ops.{module}: {msg}", flush=True)
        else:
            _imported.add(module)


def get_op(name: str) -> OpFn:
    """Resolve ``name`` to its handler, importing its module lazily."""
    if not _is_enabled(name):
        raise ValueError(f"Op {name!r} is not enabled by TASKS. Enabled ops: {list_ops()}")
    module = OP_TO_MODULE.get(name)
    if not module:
        raise ValueError(f"Unknown op {name!r}. Allowed ops: {sorted(OP_TO_MODULE)}")
    _import_module(module)
    fn = OPS_REGISTRY.get(name)
    if fn is not None:
        return fn
    registered = sorted(OPS_REGISTRY)
    if OPS_LOAD_ERRORS:
        shown = "; ".join(f"{m} => {e}" for m, e in OPS_LOAD_ERRORS[:10])
        extra = len(OPS_LOAD_ERRORS) - 10
        tail = f" (+{extra} more)" if extra > 0 else ""
        raise ValueError(
            f"Unknown or failed op {name!r}. Registered ops: {registered}. "
            f"Also saw op import errors: {shown}{tail}"
        )
    raise ValueError(f"Unknown op {name!r}. Registered ops: {registered}")


def _reset_for_tests() -> None:
    """Forget import failures so a test can re-probe (not used by the agent)."""
    with _lock:
        _failed.clear()
        del OPS_LOAD_ERRORS[:]


__all__ = [
    "OPS_REGISTRY",
    "OPS_LOAD_ERRORS",
    "OP_TO_MODULE",
    "OPT_IN_OPS",
    "BATCH_REGISTRY",
    "register_op",
    "register_batch_op",
    "get_batch_op",
    "list_ops",
    "get_op",
]
