"""Collective job execution: rank 0 leases, every rank computes its shard.

Process model (one process per GPU, ``torchrun --nproc-per-node N app.py``):
rank 0 runs the HTTP agent loop; ranks 1..N-1 sit in :func:`worker_loop`.
For a DP-capable job rank 0 calls :func:`dispatch`, which broadcasts the task
descriptor (C4) and then runs the same registered ``@dp_task`` body as every
worker. Bodies do their local (collective-free) work first; the per-rank
errors are then exchanged, so a failure on ANY rank fails the job on rank 0
with that rank's id in the message instead of hanging the others in a
collective. ``MI355X_FAULT=rank:K[:stage[:times]]`` injects a
failure on rank K for tests; a ``:device`` kind raises a HIP-style device
fault, which drops that rank from the DP group (elastic shrink, SURVEY.md
§5.3) while the job that hit it fails and names the rank.

Registered bodies: ``map_classify_csv`` (C2 all-gather of top-k),
``risk_accumulate`` (C3 all-reduce of {count,sum,min,max}) and
``map_summarize`` (C5 all-gather of generated token ids).
"""
from __future__ import annotations

import os
import threading
import time
import traceback
from typing import Any, Callable, Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..utils.trace import DeviceStages, span
from . import dp, watchdog
from .dp import all_gather_rows, broadcast_task, comm_device, is_dist, members, split_range, world

_TASKS: Dict[str, Callable[[Dict[str, Any]], Any]] = {}
_SHUTDOWN = "__shutdown__"


def dp_task(name: str):
    def wrap(fn):
        _TASKS[name] = fn
        return fn

    return wrap


def init_from_env() -> None:
    """Join the node's process group (RCCL on GPUs, gloo otherwise) with a bounded
    collective timeout (``DP_COLLECTIVE_TIMEOUT`` s), and start this rank's heartbeat."""
    if is_dist():
        return
    from datetime import timedelta

    local = int(os.getenv("LOCAL_RANK", "0"))
    timeout = timedelta(seconds=watchdog.collective_timeout())
    if torch.cuda.is_available() and os.getenv("ATPU_DP_BACKEND", "nccl") == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
    else:
        if torch.cuda.is_available():  # gloo rehearsal: ranks may share a GPU
            torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("gloo", timeout=timeout)
    watchdog.start(dist.get_rank())


_FAULT_HITS: Dict[str, int] = {}


# substrings of a HIP/HSA device fault (vs. an ordinary Python error of the op)
FAULT_MARKERS = ("hipError", "HIP error", "HSA_STATUS_ERROR", "illegal memory access", "device-side assert",
                 "GPU Hang", "Memory access fault")


def is_device_fault(msg: str) -> bool:
    return any(m in msg for m in FAULT_MARKERS)


class DPError(RuntimeError):
    """A DP job failed on one or more ranks; the message names each rank.

    Ops must not turn this into a soft result (``map_classify``'s fallback
    stub): the agent has to see it to mark faulted devices unhealthy."""


class LeftGroup(DPError):
    """This rank's device faulted and it was dropped from the DP group."""


def maybe_inject_fault(stage: str) -> None:
    """``MI355X_FAULT=rank:K[:stage[:times[:device]]]`` raises on global rank K
    (optionally only at ``stage``, only the first ``times`` times — later tasks
    succeed, so tests can check that the DP group survives — and as a device
    fault with ``:device``)."""
    spec = os.getenv("MI355X_FAULT", "")
    if not spec.startswith("rank:"):
        return
    rank = dist.get_rank() if is_dist() else 0
    parts = spec.split(":")
    if int(parts[1]) != rank or (len(parts) >= 3 and parts[2] not in ("", stage)):
        return
    if len(parts) >= 4 and parts[3]:
        n = _FAULT_HITS.get(stage, 0)
        if n >= int(parts[3]):
            return
        _FAULT_HITS[stage] = n + 1
    kind = parts[4] if len(parts) >= 5 else ""
    if kind == "device":
        raise RuntimeError(f"hipErrorLaunchFailure: injected device fault ({spec}) at {stage}")
    if kind == "kill":  # the process dies mid-job (OOM killer, abort, SIGKILL)
        import signal

        os.kill(os.getpid(), signal.SIGKILL)
    if kind == "hang":  # a wedged rank: alive, heartbeat running, never reaches the next collective
        time.sleep(1e6)
    raise RuntimeError(f"injected fault ({spec}) at {stage}")


_ERR_TYPES = {"ValueError": ValueError, "TypeError": TypeError, "KeyError": KeyError,
              "FileNotFoundError": FileNotFoundError}


def _check_errors(err: str, extra: Any = None) -> Optional[list]:
    """Exchange per-rank errors (``"Type: message"``) so every rank fails together.

    If EVERY rank failed with the same input-validation error (a bad payload is
    bad everywhere) it is re-raised with its own type and message, keeping the
    single-process op's contract; otherwise a RuntimeError names each rank.

    ``extra``: a small per-rank value carried by the SAME object exchange (e.g. the
    rank's row count for the C2 all-gather, which then needs no count collective of
    its own); returns every rank's ``extra`` in group order (None outside a group:
    ``[extra]``).
    """
    if not is_dist():
        if err:
            raise RuntimeError(err)
        return [extra]
    rank, ws = world()
    errs = [None] * ws
    with watchdog.collective("error exchange"):
        dist.all_gather_object(errs, (err, extra), group=dp.group())
    extras = [e[1] for e in errs]
    errs = [e[0] for e in errs]
    glob = members()  # group index -> global rank (errors name global ranks)
    bad = [(glob[r], e) for r, e in enumerate(errs) if e]
    if not bad:
        return extras
    if len(bad) == ws and len(set(e for _, e in bad)) == 1:
        typ, _, msg = bad[0][1].partition(": ")
        if typ in _ERR_TYPES:
            raise _ERR_TYPES[typ](msg)
    msg = "; ".join(f"rank {r}: {e}" for r, e in bad)
    faulted = [r for r, e in bad if is_device_fault(e)]
    if faulted and os.getenv("ATPU_ELASTIC", "1") != "0" and dp.shrink(faulted):
        if dist.get_rank() in faulted:
            raise LeftGroup(msg)
        msg += f" (dropped from the DP group: ranks {faulted}; DP world now {len(members())})"
    raise DPError(msg)


def _err_str(exc: BaseException) -> str:
    return f"{type(exc).__name__}: {exc}"


_CTX = threading.local()


def in_task() -> bool:
    """True while this rank executes a dispatched DP task body (every rank of
    the group runs the same body, so collectives inside it pair up)."""
    return getattr(_CTX, "depth", 0) > 0


def run_collective(name: str, payload: Dict[str, Any]) -> Any:
    fn = _TASKS[name]
    _CTX.depth = getattr(_CTX, "depth", 0) + 1
    watchdog.progress(f"run {name}")
    try:
        return fn(payload)
    finally:
        _CTX.depth -= 1
        watchdog.progress("idle")


def load_collectively(local: Callable[[], Any], collective: Callable[[Any], Any],
                      post: Optional[Callable[[Any], Any]] = None) -> Any:
    """Model-load protocol of a DP task: no rank enters the C1 broadcast
    unless every rank is ready for it.

    1. ``local()`` on every rank: rank 0 builds the source weights on the
       host (seeded init or a safetensors load), the others allocate the
       destination; either may raise (bad path, missing tensor, HBM OOM).
    2. Errors are exchanged (:func:`_check_errors`): one failure fails the
       job on EVERY rank before any collective is issued, so a rank that
       leaves early never pairs a later broadcast with a stale one.
    3. ``collective(state)``: the broadcast itself, reached by all or none.
    4. ``post(result)`` (engine / graph build, local) with a second exchange,
       so a per-rank OOM there also fails every rank together.

    Outside a process group it is just ``post(collective(local()))`` with the
    error raised directly.
    """
    err, state = "", None
    try:
        state = local()
    except Exception as exc:
        err = _err_str(exc)
        if not is_dist():
            raise
    _check_errors(err)
    out = collective(state)
    if post is None:
        return out
    err, res = "", None
    try:
        res = post(out)
    except Exception as exc:
        err = _err_str(exc)
        if not is_dist():
            raise
    _check_errors(err)
    return res


def _announce() -> None:
    """Rank 0: flag task ``seq`` in the store; idle workers wait on that key, not in a
    collective, so an idle gap between jobs never trips the collective timeout."""
    seq = watchdog.next_task()
    st = watchdog._get_store()
    if st is not None:
        st.set(f"task/{seq}", "1")


def _await_task() -> bool:
    """Worker: block until rank 0 announces the next task; False if rank 0 is gone."""
    from datetime import timedelta

    seq = watchdog.next_task()
    st = watchdog._get_store()
    if st is None:
        return True
    while True:
        try:
            st.wait([f"task/{seq}"], timedelta(seconds=5))
            return True
        except Exception:
            pid = watchdog._get("pid/0")
            if pid is not None and not watchdog._pid_alive(int(pid)):
                return False


def dispatch(name: str, payload: Dict[str, Any]) -> Any:
    """Rank 0: broadcast ``(name, payload)`` then execute it with every rank."""
    if is_dist():
        _announce()
        broadcast_task({"op": name, "payload": payload})
    return run_collective(name, payload)


def worker_loop() -> int:
    """Ranks != 0: execute broadcast task descriptors until shutdown."""
    rank, _ = world()
    print(f"[agent-mi355x] dp worker rank={rank} ready", flush=True)
    while True:
        if not _await_task():
            print(f"[agent-mi355x] dp worker rank={rank}: rank 0 is gone; exiting", flush=True)
            return watchdog.EXIT_RANK_LOST
        desc = broadcast_task(None)
        if not isinstance(desc, dict) or desc.get("op") == _SHUTDOWN:
            break
        try:
            run_collective(desc["op"], desc["payload"])
        except LeftGroup as exc:
            print(f"[agent-mi355x] dp worker rank={rank} left the DP group after a device fault: {exc}", flush=True)
            break
        except Exception as exc:  # rank 0 reports; keep serving
            print(f"[agent-mi355x] dp worker rank={rank} task {desc.get('op')} failed: {exc}", flush=True)
    if is_dist():
        dist.destroy_process_group()
    return 0


def shutdown_workers() -> None:
    if is_dist() and world()[0] == 0:
        _announce()
        broadcast_task({"op": _SHUTDOWN})


# ------------------------------------------------------------ health
@dp_task("health_check")
def health_task(payload: Dict[str, Any]) -> Any:
    """Every rank probes ONLY its own GPU (no HIP context on a peer's device);
    rank 0 merges the per-rank answers into the node view it advertises."""
    from ..runtime import health

    if torch.cuda.is_available():
        res = health.check(probe=bool(payload.get("probe", True)), only=[torch.cuda.current_device()])
    else:
        res = {"ok": False, "devices": [], "healthy": [], "unhealthy": {}, "error": "no ROCm device visible"}
    from .placement import current_plan, host_threads

    plan = current_plan()
    try:
        ncpu = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        ncpu = os.cpu_count() or 0
    # this rank's row of the node's rank table: its device and host placement (placement.py)
    res["rank_info"] = {"rank": dist.get_rank() if is_dist() else 0, "local_rank": int(os.getenv("LOCAL_RANK", "0")),
                        "device": torch.cuda.current_device() if torch.cuda.is_available() else None,
                        "numa": plan["numa"] if plan else None, "ncpus": ncpu, "host_threads": host_threads(),
                        "placement": plan["source"] if plan else "unplaced"}
    parts = [res]
    if is_dist():
        parts = [None] * world()[1]
        with watchdog.collective("health gather"):
            dist.all_gather_object(parts, res, group=dp.group())
    if world()[0] != 0:
        return None
    return health.set_last(health.merge(parts))


# ------------------------------------------------------------ map_classify
def _open_table(path: str):
    from ..io.csv import open_csv

    return open_csv(path)


@dp_task("map_classify_csv")
def classify_csv_task(payload: Dict[str, Any]) -> Any:
    from ops._gpu_runtime import get_gpu_handle, get_model_path  # agent-level registry

    rank, ws = world()
    timing: Dict[str, float] = {}
    # model load is itself collective (C1 broadcast, errors exchanged before it), on every rank
    with span("load_ms", timing):
        h = get_gpu_handle(get_model_path(payload.get("model_path")))
    if getattr(h, "fresh", False):  # an LRU miss: this job paid the cold load (phases)
        h.fresh = False
        timing["cold_load"] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in h.load_ms.items()}
    err, idx, sc, meta = "", None, None, {}
    try:
        start = int(payload.get("start_row", 0))
        size = int(payload.get("shard_size", 100))
        if start < 0 or size <= 0:
            raise ValueError("start_row must be >= 0 and shard_size > 0")
        table = _open_table(payload["source_uri"])
        col = table.native.column_index(str(payload.get("text_column", "text")))
        if col < 0:
            raise ValueError(f"text_column {payload.get('text_column', 'text')!r} not in header {table.header}")
        total = max(0, min(size, table.num_rows - start))
        s_r, n_r = split_range(start, total, ws, rank)
        maybe_inject_fault("classify")
        with span("classify_ms", timing):
            idx, sc, st = h.engine.classify_table(table.native, s_r, n_r, col,
                                                  stage_timing=payload.get("timing", "host") == "device")
        timing.update({k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.timing_ms.items()})
        meta = {"start_row": start, "end_row": start + total, "world": ws}
    except Exception as exc:
        err = f"{type(exc).__name__}: {exc}"
        if os.getenv("ATPU_DEBUG"):
            traceback.print_exc()
    # one object exchange: the errors AND every rank's row count (the C2 all-gather below
    # needs no count collective and no host sync of its own)
    counts = _check_errors(err, int(idx.shape[0]) if idx is not None else 0)
    dev_t = idx is not None and idx.is_cuda
    ev = DeviceStages.event if dev_t else (lambda *a: None)
    g0 = ev()
    with span("host_allgather_ms", timing):
        idx, sc = all_gather_rows(idx, sc, counts=counts)
    g1 = ev()
    if rank != 0:
        return None
    with span("host_d2h_ms", timing):
        idx_h, sc_h = idx.cpu(), sc.cpu()
    g2 = ev()
    if dev_t:
        g2.synchronize()
        timing["device_allgather_ms"] = round(g0.elapsed_time(g1), 3)
        timing["device_d2h_ms"] = round(g1.elapsed_time(g2), 3)
    meta["timing_ms"] = timing
    from ops.map_classify import csv_result

    return csv_result(h, idx_h, sc_h, meta, payload)


@dp_task("map_classify_rows")
def classify_rows_task(payload: Dict[str, Any]) -> Any:
    """``input`` (one pre-tokenized row: rank 0 computes it) and ``texts``
    (rows split over the ranks, top-k all-gathered, C2) forms of map_classify.
    The model load is collective on every rank either way."""
    from ops import map_classify as mc
    from ops._gpu_runtime import get_gpu_handle, get_model_path

    rank, ws = world()
    h = get_gpu_handle(get_model_path(payload.get("model_path")))
    op, t0 = payload.get("_op", mc.OP_NAME), float(payload.get("_t0", time.time()))
    if "input" in payload:
        return mc.classify_ids(h, payload, op, t0) if rank == 0 else None
    texts = mc.check_texts(payload)  # same payload on every rank: same outcome, no exchange needed
    k = max(1, min(int(payload.get("topk", 5)), h.cfg.num_labels))
    err, idx, sc = "", None, None
    try:
        s_r, n_r = split_range(0, len(texts), ws, rank)
        maybe_inject_fault("classify")
        res = h.engine.classify_texts(texts[s_r:s_r + n_r], k)
        idx, sc = res.idx[:, :k].contiguous(), res.score[:, :k].contiguous()
    except Exception as exc:
        err = _err_str(exc)
    counts = _check_errors(err, int(idx.shape[0]) if idx is not None else 0)
    idx, sc = all_gather_rows(idx, sc, counts=counts)
    if rank != 0:
        return None
    return mc.texts_result(h, idx.cpu(), sc.cpu(), payload, ws)


@dp_task("map_classify_batch")
def classify_batch_task(payload: Dict[str, Any]) -> Any:
    """Several ``input``/``texts`` jobs of one lease (same model): one collective model
    load, then :func:`ops.map_classify.classify_batch` on every rank."""
    from ops import map_classify as mc
    from ops._gpu_runtime import get_gpu_handle, get_model_path

    rank, ws = world()
    payloads = payload["payloads"]
    h = get_gpu_handle(get_model_path(payloads[0].get("model_path")))
    return mc.classify_batch(h, payloads, rank, ws)


# ---------------------------------------------------------- risk_accumulate
def _local_values(payload: Dict[str, Any], rank: int, ws: int) -> Tuple[torch.Tensor, int]:
    """This rank's slice of a ``values`` / ``items`` payload, as fp64 (CSV payloads stream
    through :func:`csv_stats` instead and are never materialised)."""
    from ops.risk_accumulate import gather_array  # same validation/messages as the CPU op (native parse)

    vals = gather_array(payload)
    s_r, n_r = split_range(0, len(vals), ws, rank)
    return torch.from_numpy(vals[s_r:s_r + n_r].copy()), len(vals)


def csv_stats(payload: Dict[str, Any], rank: int, ws: int, device: Any = "auto"):
    """This rank's share of a CSV ``risk_accumulate``: streamed in chunks (runtime/risk.py),
    never materialised. -> (fp64 [count, sum, min, max] on the CPU, stream info).

    ``device="auto"``: the GPU (:func:`risk_device`) only for a shard of at least
    ``gpu_min_rows()`` rows, decided BEFORE anything touches HIP: a small shard reduces on the
    host without creating a GPU context."""
    from ..runtime.risk import column_stats, gpu_min_rows

    table = _open_table(payload["source_uri"])
    col = table.native.column_index(str(payload.get("field", "risk")))
    if col < 0:
        raise ValueError(f"field {payload.get('field', 'risk')!r} not in header {table.header}")
    start = int(payload.get("start_row", 0))
    total = max(0, min(int(payload.get("shard_size", table.num_rows)), table.num_rows - start))
    s_r, n_r = split_range(start, total, ws, rank)
    if isinstance(device, str):  # "auto"
        device = risk_device() if n_r >= gpu_min_rows() else None
    return column_stats(table.native, s_r, n_r, col, device)


def risk_device() -> Optional[torch.device]:
    """The GPU the risk reduce runs on (``RISK_DEVICE=cpu`` keeps it on the host)."""
    if os.getenv("RISK_DEVICE", "auto").strip().lower() == "cpu" or not torch.cuda.is_available():
        return None
    return torch.device("cuda", torch.cuda.current_device())


@dp_task("risk_accumulate")
def risk_task(payload: Dict[str, Any]) -> Any:
    from ..ops.reduce import reduce_stats_tensor, stats_dict

    t0 = time.perf_counter()
    rank, ws = world()
    err, stats = "", torch.tensor([0.0, 0.0, float("inf"), float("-inf")], dtype=torch.float64)
    try:
        maybe_inject_fault("risk")
        if "source_uri" in payload:
            stats, _ = csv_stats(payload, rank, ws)
        else:
            x, _ = _local_values(payload, rank, ws)
            if torch.cuda.is_available():
                dev = torch.device("cuda", torch.cuda.current_device())
                x = x.to(dev, non_blocking=True)
            if x.numel():
                stats = reduce_stats_tensor(x)
    except Exception as exc:
        err = f"{type(exc).__name__}: {exc}"
    _check_errors(err)
    if is_dist():
        cdev = comm_device()
        s = stats.to(cdev)
        sums = s[:2].clone()
        ext = torch.stack([s[3], -s[2]])  # max, -min -> one MAX all-reduce
        nc = dp.native_comm(cdev)
        with watchdog.collective("risk all-reduce"):
            if nc is not None:
                nc.all_reduce(sums, "sum")
                nc.all_reduce(ext, "max")
                nc.wait("risk all-reduce")
            else:
                dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=dp.group())
                dist.all_reduce(ext, op=dist.ReduceOp.MAX, group=dp.group())
        stats = torch.stack([sums[0], sums[1], -ext[1], ext[0]]).cpu()
    else:
        stats = stats.cpu()
    if rank != 0:
        return None
    out = stats_dict(stats.tolist())
    out["compute_time_ms"] = (time.perf_counter() - t0) * 1000.0
    out["dp_world_size"] = ws
    return out


# ------------------------------------------------------------ map_summarize
@dp_task("map_summarize")
def summarize_task(payload: Dict[str, Any]) -> Any:
    """Each rank beam-searches its contiguous shard of the documents; the
    int32 token ids ``[docs_r, max_length]`` (-1 padded) are all-gathered to
    rank 0 (C5), which detokenizes. Reference: ``ops/map_summarize.py:46-68``
    (one document per call, CPU)."""
    import ops.map_summarize as ms

    rank, ws = world()
    timing: Dict[str, float] = {}
    with span("load_ms", timing):
        eng = ms._init_engine()  # first call: C1 broadcast of the weights
    texts = payload["texts"]
    gen = ms._gen_config(payload)
    err, steps = "", 0
    seqs = torch.full((0, gen.max_length), -1, dtype=torch.int32)
    maps = None
    if rank == 0 and eng.device.type == "cuda":  # detokenization maps built while the GPUs decode
        from ..runtime.summarize import _host_pool

        maps = _host_pool().submit(eng.word_maps, texts)
    try:
        s_r, n_r = split_range(0, len(texts), ws, rank)
        maybe_inject_fault("summarize")
        if n_r:
            with span("generate_ms", timing):
                res = eng.generate_ids(texts[s_r:s_r + n_r], gen)
            steps = res.steps
            seqs = torch.full((n_r, gen.max_length), -1, dtype=torch.int32)
            for i, sq in enumerate(res.sequences):
                seqs[i, :len(sq)] = torch.tensor(sq[:gen.max_length], dtype=torch.int32)
    except Exception as exc:
        err = f"{type(exc).__name__}: {exc}"
        if os.getenv("ATPU_DEBUG"):
            traceback.print_exc()
    counts = _check_errors(err, int(seqs.shape[0]))
    with span("allgather_ms", timing):
        (seqs,) = all_gather_rows(seqs, counts=counts)
    if rank != 0:
        return None
    rows = [[int(t) for t in r if t >= 0] for r in seqs.cpu().tolist()]
    if maps is not None:
        summaries = [eng.detokenize(s, m) for s, m in zip(rows, maps.result())]
    else:
        summaries = eng.detokenize_all(texts, rows)
    return ms.result(bool(payload.get("texts_mode", True)), summaries, steps, timing,
                     float(payload.get("t0", time.time())), dp_world_size=ws)
