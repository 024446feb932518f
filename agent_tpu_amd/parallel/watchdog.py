"""Dead- and hung-rank detection for the DP agent.

The reference has no failure detection beyond the controller's lease TTL
(``/root/reference/app.py:166``). Here one process drives each GPU, so a rank
can die (SIGKILL, OOM, a HIP fault that aborts) or hang (a wedged kernel)
mid-job. Rank 0, which owns the HTTP loop, must then fail the in-flight jobs
naming that rank instead of blocking in a collective until a backend timeout
tears the process down without a result.

Mechanism (all through the job's c10d TCPStore, no extra sockets):

* every rank publishes its PID and a heartbeat (``atpu/hb/<rank>``, every
  ``DP_HEARTBEAT_SEC``) plus a progress marker ``atpu/prog/<rank>`` =
  ``"<task seq>:<stage>"`` at every stage of a DP task;
* rank 0 marks when it enters a collective (:func:`collective`);
* rank 0's :class:`Watchdog` thread declares ranks lost when their process is
  gone (the node is shared, so PID liveness is exact and immediate), their
  heartbeat is older than ``DP_HEARTBEAT_TIMEOUT``, or rank 0 has sat in one
  collective for ``0.8 * DP_COLLECTIVE_TIMEOUT`` — the ranks whose progress
  marker is behind rank 0's are named (before RCCL's own watchdog would abort
  the process at the full timeout);
* a collective that raises on rank 0 (gloo: peer connection closed / timed
  out) is re-raised as :class:`RankLost` naming the same ranks.

The agent reacts by posting ``failed`` for its in-flight jobs and exiting
non-zero, so the launcher (``torchrun --max-restarts``) restarts the group in
fresh processes (never ``exec``).
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from typing import Callable, List, Optional, Tuple

import torch.distributed as dist

HB_SEC = float(os.getenv("DP_HEARTBEAT_SEC", "1.0"))
HB_TIMEOUT = float(os.getenv("DP_HEARTBEAT_TIMEOUT", "15"))
COLLECTIVE_TIMEOUT = float(os.getenv("DP_COLLECTIVE_TIMEOUT", "120"))
EXIT_RANK_LOST = 3


def collective_timeout() -> float:
    return float(os.getenv("DP_COLLECTIVE_TIMEOUT", str(COLLECTIVE_TIMEOUT)))


class RankLost(RuntimeError):
    """A DP rank died or hung; the message names it. Fatal for the DP group."""


_store = None
_rank = 0
_seq = 0
_in_collective: Optional[Tuple[float, str]] = None
_hb_thread: Optional[threading.Thread] = None
_stop = threading.Event()


def _get_store():
    global _store
    if _store is None and dist.is_initialized():
        try:
            from torch.distributed.distributed_c10d import _get_default_store

            _store = dist.PrefixStore("atpu/", _get_default_store())
        except Exception:
            _store = None
    return _store


def _set(key: str, val: str) -> None:
    st = _get_store()
    if st is not None:
        try:
            st.set(key, val)
        except Exception:
            pass


def _get(key: str) -> Optional[str]:
    st = _get_store()
    if st is None:
        return None
    try:
        if not st.check([key]):
            return None
        return st.get(key).decode()
    except Exception:
        return None


def start(rank: int) -> None:
    """Publish this rank's PID and start its heartbeat thread."""
    global _rank, _hb_thread
    _rank = rank
    if _get_store() is None or _hb_thread is not None:
        return
    _set(f"pid/{rank}", str(os.getpid()))
    _set(f"prog/{rank}", "0:init")

    def beat():
        while not _stop.wait(HB_SEC):
            _set(f"hb/{rank}", repr(time.time()))

    _set(f"hb/{rank}", repr(time.time()))
    _hb_thread = threading.Thread(target=beat, name=f"atpu-hb-{rank}", daemon=True)
    _hb_thread.start()


def stop() -> None:
    _stop.set()


def next_task() -> int:
    global _seq
    _seq += 1
    return _seq


def active() -> bool:
    """True once :func:`start` ran on this rank (the agent's DP process model)."""
    return _hb_thread is not None


def progress(stage: str) -> None:
    if _hb_thread is None:  # not an agent rank (bench / tests): no store traffic
        return
    _set(f"prog/{_rank}", f"{_seq}:{stage}")


@contextlib.contextmanager
def collective(stage: str):
    """Bracket a collective: progress marker, rank-0 wait clock, named failure."""
    global _in_collective
    if _hb_thread is None:  # watchdog not running on this rank: a plain collective
        yield
        return
    progress(f"enter {stage}")
    if _rank == 0:
        _in_collective = (time.monotonic(), stage)
    try:
        yield
    except RankLost:
        raise
    except Exception as exc:
        if _rank == 0 and _get_store() is not None:
            lost = diagnose()
            if lost:
                raise RankLost(describe(lost) + f" ({stage}: {type(exc).__name__}: {str(exc)[:200]})") from exc
        raise
    finally:
        if _rank == 0:
            _in_collective = None
        progress(f"done {stage}")


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:  # a killed child stays a zombie until the launcher reaps it
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] not in ("Z", "X")
    except OSError:
        return True


def diagnose(hung_after: Optional[float] = None) -> List[Tuple[int, str]]:
    """Members of the active DP group that are gone (dead PID / stale heartbeat) or,
    with ``hung_after``, behind rank 0. Ranks already dropped (elastic shrink after a
    device fault, :func:`agent_tpu_amd.parallel.dp.shrink`) are not watched."""
    from .dp import members

    lost: List[Tuple[int, str]] = []
    now = time.time()
    mine = _get(f"prog/{_rank}") or ""
    for r in members():
        if r == _rank:
            continue
        pid = _get(f"pid/{r}")
        if pid is not None and not _pid_alive(int(pid)):
            lost.append((r, f"process died (pid {pid})"))
            continue
        hb = _get(f"hb/{r}")
        if hb is not None and now - float(hb) > HB_TIMEOUT:
            lost.append((r, f"no heartbeat for {now - float(hb):.1f} s"))
            continue
        if hung_after is not None:
            prog = _get(f"prog/{r}") or "?"
            if prog != mine:
                lost.append((r, f"hung at task/stage {prog!r} while rank {_rank} waited "
                                f"{hung_after:.1f} s in {mine!r}"))
    return lost


def describe(lost: List[Tuple[int, str]]) -> str:
    return "; ".join(f"rank {r}: {why}" for r, why in lost) + " (DP rank lost)"


class Watchdog:
    """Rank-0 monitor thread: calls ``on_lost(message)`` once when a rank is lost."""

    def __init__(self, on_lost: Callable[[str], None], interval: float = 0.5):
        self.on_lost, self.interval = on_lost, interval
        self._t = threading.Thread(target=self._run, name="atpu-dp-watchdog", daemon=True)
        self.fired = False

    def start(self) -> "Watchdog":
        self._t.start()
        return self

    def _run(self) -> None:
        limit = 0.8 * collective_timeout()
        while not _stop.wait(self.interval):
            ic = _in_collective
            waited = time.monotonic() - ic[0] if ic is not None else None
            lost = diagnose(hung_after=waited if waited is not None and waited > limit else None)
            if lost:
                self.fired = True
                self.on_lost(describe(lost))
                return
