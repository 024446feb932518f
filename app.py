#!/usr/bin/env python3
"""MI355X job agent: lease -> execute -> report.

Wire protocol and env contract of the reference agent
(``/root/reference/app.py``): ``POST /v1/leases`` with
``{agent, capabilities:{ops}, max_tasks, timeout_ms, labels, worker_profile,
metrics}`` (ref ``app.py:161-195``); ``POST /v1/results`` with
``{lease_id, job_id, job_epoch, status, result, error}`` (ref ``:198-218``);
error objects ``{type, message, trace}`` (ref ``:288-294``); exit code 2 when
``TASKS`` is empty, 0 after SIGINT/SIGTERM (ref ``:245-316``).

Fixes over the reference:

* ops are resolved through the ``ops`` registry / ``ops_loader`` (the
  reference's ``app.py`` had a private two-entry table, §2.4.1-2);
* the worker profile is built dynamically by ``worker_sizing`` (AMD GPUs,
  HBM-derived batch sizing) plus the reference's ``tier``/``limits`` (§2.4.3);
* EVERY task of a multi-task lease is executed and resulted (§2.4.8);
* one keep-alive HTTP connection instead of a TCP connect per request (§2.4.11);
* failed result posts get a bounded retry on transport/5xx errors, never on
  4xx (a 409 stale epoch is final); ``job_epoch`` is passed through verbatim;
* metrics add GPU/HBM use, completed jobs and a rolling rows/s (§5.5);
* the next lease is taken while the current batch runs and results are posted by a
  background thread (``LEASE_PREFETCH`` / ``RESULT_POST_ASYNC``, both on by default; 0 restores
  the reference's serial order), so neither HTTP round trip sits between two jobs' GPU work.

Data parallel: launched under ``torchrun`` (WORLD_SIZE>1), rank 0 runs this
loop and the other ranks run :func:`agent_tpu_amd.parallel.dp_ops.worker_loop`,
executing their shard of every DP-capable job (map_classify, risk_accumulate).
"""
from __future__ import annotations

import json
import os
import signal
import socket
import sys
import threading
import time
import traceback
from collections import deque
from typing import Any, Deque, Dict, List, Optional, Tuple

try:
    import requests
except Exception:  # pragma: no cover
    requests = None

try:
    import psutil  # type: ignore
except Exception:  # pragma: no cover
    psutil = None

LOG = "[agent-mi355x]"

# rank-process environment (RCCL IPC mode), applied before any GPU use however the agent
# was launched (plain, or one rank per GPU under torch.distributed.run): see
# agent_tpu_amd.parallel.launch.RANK_ENV_DEFAULTS (a stdlib-only module)
from agent_tpu_amd.parallel.launch import ensure_rank_env  # noqa: E402

ensure_rank_env()
# a job's result must not depend on which other jobs share its device batch (lease batching,
# in-flight batching, DP shards): batch-invariant kernel selection unless the operator opts out
os.environ.setdefault("ATPU_BATCH_INVARIANT", "1")

# ------------------------------------------------------------------ config
# identical names and defaults to the reference (app.py:21-41)
CONTROLLER_URL = os.getenv("CONTROLLER_URL", "").rstrip("/") or "http://10.11.12.54:8080"
AGENT_NAME = os.getenv("AGENT_NAME", socket.gethostname())
HTTP_TIMEOUT_SEC = float(os.getenv("HTTP_TIMEOUT_SEC", "10"))
IDLE_SLEEP_SEC = float(os.getenv("IDLE_SLEEP_SEC", "0.25"))
MAX_TASKS = int(os.getenv("MAX_TASKS", "1"))
LEASE_TIMEOUT_MS = int(os.getenv("LEASE_TIMEOUT_MS", "3000"))
ERROR_LOG_EVERY_SEC = float(os.getenv("ERROR_LOG_EVERY_SEC", "10"))
ERROR_BACKOFF_SEC = float(os.getenv("ERROR_BACKOFF_SEC", "1.0"))
TASKS_RAW = os.getenv("TASKS", "echo,map_classify_tpu")
AGENT_LABELS_RAW = os.getenv("AGENT_LABELS", "")
# new knobs
RESULT_RETRIES = int(os.getenv("RESULT_RETRIES", "2"))
# same-op jobs of one lease run as ONE device batch (map_summarize docs, map_classify rows)
LEASE_BATCH = os.getenv("LEASE_BATCH", "1").strip().lower() not in ("0", "false", "no", "off")
# post results from a background thread (FIFO, bounded): the next job's device work overlaps
# the HTTP post of the previous result (and the controller's parse of it). 0 = the reference's
# strictly serial lease -> execute -> post order.
RESULT_POST_ASYNC = os.getenv("RESULT_POST_ASYNC", "1").strip().lower() in ("1", "true", "yes", "on")
# lease the next task batch while the current one runs (one lease ahead, own connection): the
# lease round trip leaves the critical path between jobs. 0 = lease only when idle (reference).
LEASE_PREFETCH = os.getenv("LEASE_PREFETCH", "1").strip().lower() in ("1", "true", "yes", "on")
# lease size this agent can batch well; advertised in worker_profile.limits (MAX_TASKS stays the request)
MAX_BATCH_TASKS = int(os.getenv("MAX_BATCH_TASKS", "1024"))
# with RESULT_POST_ASYNC: results that queue up while the poster is busy go out pipelined on one
# keep-alive connection (PipelinedPoster); 0 = one request / response round trip per result
RESULT_PIPELINE = os.getenv("RESULT_PIPELINE", "1").strip().lower() in ("1", "true", "yes", "on")
METRICS_REFRESH_SEC = float(os.getenv("METRICS_REFRESH_SEC", "0.25"))
# a lease taken ahead (LEASE_PREFETCH) but not started when SIGINT/SIGTERM arrives: "ttl" (default:
# not run, nothing posted, the controller re-leases it after LEASE_TIMEOUT_MS) or "fail" (posted
# failed with error type "Shutdown")
SHUTDOWN_AHEAD = os.getenv("SHUTDOWN_AHEAD", "ttl").strip().lower()
# in-flight (continuous) execution: up to this many leased jobs are held at once, leased by a
# helper thread (pipelined HTTP/1.1 lease requests) while the device runs; batchable ops run the
# jobs queued so far as the next device batch, map_summarize jobs join the running beam searches
# at their next decode step (ops.register_stream_op). "auto" (default): sized from the enabled GPU
# ops' batch sizes and LEASE_TIMEOUT_MS on a GPU agent, 1 (the serial loop) otherwise; 0/1 = the
# serial lease -> run -> post loop. Controller-visible: the agent holds up to this many leases.
INFLIGHT_DEPTH_RAW = os.getenv("INFLIGHT_DEPTH", "auto").strip().lower()
# lease requests sent back to back on one keep-alive connection (at most) per round trip
LEASE_PIPELINE_MAX = int(os.getenv("LEASE_PIPELINE_MAX", "64"))
# auto in-flight depth: hold at most what the measured completion rate finishes within this fraction of
# the lease TTL (never less than a third of the sized depth, nor more than all of it; all of it until
# completions are measured)
INFLIGHT_TTL_FRACTION = float(os.getenv("INFLIGHT_TTL_FRACTION", "0.6"))
# a single job's result is held back for a grouped post only behind jobs shorter than this
DEFER_MAX_JOB_SEC = float(os.getenv("DEFER_MAX_JOB_SEC", "0.001"))
FAIL_ON_NOT_OK = os.getenv("FAIL_ON_NOT_OK", "0").strip().lower() in ("1", "true", "yes")

_running = True
_last_log: Dict[str, float] = {}
EXIT_RANK_LOST = 3  # a DP rank died or hung: restart the group (torchrun --max-restarts)


def parse_labels(raw: str) -> Dict[str, Any]:
    """``"k=v,flag,x=1=2"`` -> ``{"k": "v", "flag": True, "x": "1=2"}`` (ref app.py:49-63)."""
    labels: Dict[str, Any] = {}
    for part in (raw or "").split(","):
        part = part.strip()
        if not part:
            continue
        key, sep, val = part.partition("=")
        labels[key.strip()] = val.strip() if sep else True
    return labels


def capabilities(raw: str) -> List[str]:
    """Comma list -> de-duplicated names in first-seen order (ref app.py:86-96)."""
    seen: Dict[str, None] = {}
    for tok in (raw or "").split(","):
        tok = tok.strip()
        if tok:
            seen.setdefault(tok, None)
    return list(seen)


def log_every(key: str, msg: str) -> None:
    """Print ``msg`` at most once per ERROR_LOG_EVERY_SEC for ``key``."""
    now = time.time()
    if now - _last_log.get(key, 0.0) >= ERROR_LOG_EVERY_SEC:
        _last_log[key] = now
        print(msg, flush=True)


CAPS_LIST = capabilities(TASKS_RAW)
BASE_LABELS = parse_labels(AGENT_LABELS_RAW)


# ----------------------------------------------------------------- metrics
class Metrics:
    """Piggy-backed on every lease (ref app.py:74-83 keys + GPU/throughput)."""

    def __init__(self) -> None:
        self.jobs_completed = 0
        self.jobs_failed = 0
        self._rows: List[Tuple[float, int]] = []
        self._lock = threading.Lock()
        self._sampled: Optional[Dict[str, Any]] = None
        self._sampled_at = 0.0

    def job_done(self, ok: bool, result: Any) -> None:
        with self._lock:
            if ok:
                self.jobs_completed += 1
            else:
                self.jobs_failed += 1
            rows = result.get("row_count") if isinstance(result, dict) and ok else None
            if isinstance(rows, int) and result.get("rows_per_sec") is not None:
                self._rows.append((time.time(), rows))
                cut = time.time() - 60.0
                self._rows = [r for r in self._rows if r[0] >= cut]

    def rows_per_sec(self) -> float:
        with self._lock:
            if not self._rows:
                return 0.0
            span = max(1.0, time.time() - self._rows[0][0])
            return sum(n for _, n in self._rows) / span

    def snapshot(self) -> Dict[str, Any]:
        """The lease's ``metrics``. The host / GPU sampling (procfs and sysfs reads, ~1 ms per
        lease in this container: the cost of a 1-task echo lease) is refreshed at most every
        METRICS_REFRESH_SEC (default 0.25 s, the reference's idle poll); the job counters and
        rows/s are always current."""
        now = time.monotonic()
        if self._sampled is None or now - self._sampled_at >= METRICS_REFRESH_SEC:
            out: Dict[str, Any] = {}
            if psutil is not None:
                try:
                    out["cpu_util"] = float(psutil.cpu_percent(interval=None)) / 100.0
                    out["ram_mb"] = float(psutil.virtual_memory().used) / (1024 * 1024)
                except Exception:
                    out = {}
            out.update(gpu_metrics())
            self._sampled, self._sampled_at = out, now
        out = dict(self._sampled)
        out["jobs_completed"] = self.jobs_completed
        out["jobs_failed"] = self.jobs_failed
        out["rows_per_sec"] = round(self.rows_per_sec(), 2)
        return out


def gpu_metrics() -> Dict[str, Any]:
    """``gpu_util[]`` and ``hbm_used_gb[]``/``hbm_total_gb[]`` from amdgpu sysfs for
    every GPU of the node. Without sysfs, HBM of this process's
    own device only, and only if it already initialised it."""
    out: Dict[str, Any] = {}
    try:
        from worker_sizing import probe_gpu_busy

        util = probe_gpu_busy()
        if util:
            out["gpu_util"] = util
    except Exception:
        pass
    try:
        from worker_sizing import probe_vram

        vram = probe_vram()
        if vram:  # node-wide, from sysfs: no HIP context on any device
            out.update({"hbm_used_gb": [round(u / 2**30, 2) for u, _ in vram],
                        "hbm_total_gb": [round(t / 2**30, 2) for _, t in vram]})
            return out
        torch = sys.modules.get("torch")
        # only a process that already runs on its GPU (a CPU-only agent never imports torch for
        # this; torch.cuda.is_available() re-probes the runtime, ~20 ms per lease without a GPU)
        if torch is None or not torch.cuda.is_initialized():
            return out
        # no sysfs: this process's OWN device only (never a peer rank's GPU)
        i = torch.cuda.current_device()
        free_b, tot_b = torch.cuda.mem_get_info(i)
        out.update({"hbm_used_gb": [round((tot_b - free_b) / 2**30, 2)], "hbm_total_gb": [round(tot_b / 2**30, 2)],
                    "hbm_device": i})
    except Exception:
        pass
    return out


METRICS = Metrics()


# --------------------------------------------------------------- profile
GPU_OPS = {"map_classify", "map_classify_tpu", "map_summarize", "risk_accumulate"}
BATCH_OPS = {"map_classify", "map_classify_tpu", "map_summarize"}


def gpu_health(caps: List[str]) -> Optional[Dict[str, Any]]:
    """Start-up device check (arch, HBM, MFMA probe) when a GPU op is enabled."""
    if not (set(caps) & GPU_OPS) or os.getenv("GPU_DISABLED", "").strip().lower() in ("1", "true", "yes", "on"):
        return None
    if os.getenv("GPU_HEALTH_CHECK", "1").strip().lower() in ("0", "false", "no", "off"):
        return None
    try:
        import torch

        if not torch.cuda.is_available():
            return {"ok": False, "error": "no ROCm device visible"}
        from agent_tpu_amd.runtime import health

        if int(os.getenv("WORLD_SIZE", "1")) > 1:
            # DP: each rank probes its own GPU; rank 0 never touches a peer's device
            from agent_tpu_amd.parallel.dp_ops import dispatch

            return dispatch("health_check", {})
        return health.check()
    except Exception as exc:
        return {"ok": False, "error": f"{type(exc).__name__}: {exc}"}


def worker_profile(health: Optional[Dict[str, Any]] = None, caps: Optional[List[str]] = None) -> Dict[str, Any]:
    from worker_sizing import build_worker_profile

    prof = build_worker_profile()
    if health is not None and prof.get("gpu", {}).get("gpu_present"):
        prof["gpu"]["health"] = {"ok": health.get("ok", False), "healthy": health.get("healthy", []),
                                 "unhealthy": {str(k): v for k, v in health.get("unhealthy", {}).items()}}
        if health.get("ranks"):  # DP: one row per rank (device, NUMA node, cpuset size, thread budget)
            prof["gpu"]["health"]["ranks"] = health["ranks"]
        if "healthy" in health:
            # advertise only devices that passed (reduced capacity after a fault)
            prof["gpu"]["gpu_count"] = len(health["healthy"])
            prof["gpu"]["max_gpu_workers"] = len(health["healthy"])
    prof["tier"] = "mi355x" if prof.get("gpu", {}).get("gpu_present") else "cpu"
    prof["limits"] = {"max_payload_bytes": int(os.getenv("MAX_PAYLOAD_BYTES", "262144")),
                      "max_tokens": int(os.getenv("MAX_TOKENS", "2048"))}
    batchable = sorted(BATCH_OPS & set(caps or ()))
    if LEASE_BATCH and batchable:
        # a controller may lease up to this many same-op jobs at once: they run as one GPU batch
        prof.setdefault("workers", {})["max_batch_tasks"] = MAX_BATCH_TASKS
        prof["workers"]["batch_ops"] = batchable
    return prof


# ------------------------------------------------------------------- http
_JSON_HEADERS = {"Content-Type": "application/json"}


def _dumps(body: Dict[str, Any]) -> bytes:
    try:
        from agent_tpu_amd.utils.rawjson import dumps
    except Exception:  # pragma: no cover - package not importable: plain encoder
        return json.dumps(body, separators=(",", ":"), allow_nan=False).encode("utf-8")
    return dumps(body)


class Controller:
    """HTTP/JSON client of the controller (ref app.py:143-158) on ONE keep-alive
    connection (``http.client``: ~4x less per-request overhead than ``requests``,
    which matters for 1-row jobs at hundreds per lease). ``HTTP_CLIENT=requests``
    selects a ``requests.Session`` instead."""

    def __init__(self, base: str, timeout: float) -> None:
        import urllib.parse

        self.base = base
        self.timeout = timeout
        self.use_requests = os.getenv("HTTP_CLIENT", "").strip().lower() == "requests" and requests is not None
        self.http = requests.Session() if self.use_requests else None
        u = urllib.parse.urlsplit(base)
        self._https = u.scheme == "https"
        self._host, self._port = u.hostname or "localhost", u.port or (443 if self._https else 80)
        self._prefix = u.path.rstrip("/")
        self._conn = None

    def _connect(self):
        import http.client

        if self._conn is None:
            cls = http.client.HTTPSConnection if self._https else http.client.HTTPConnection
            self._conn = cls(self._host, self._port, timeout=self.timeout)
            return self._conn, True
        return self._conn, False

    def _drop(self) -> None:
        if self._conn is not None:
            try:
                self._conn.close()
            except Exception:
                pass
            self._conn = None

    def post(self, path: str, body: Dict[str, Any]) -> Tuple[int, Any]:
        url = self.base + path
        try:
            # compact separators (a 8192-row classify result is ~20 % smaller than requests' json=);
            # natively pre-encoded values (RawJSON: classify rows / columns) are spliced in verbatim
            data = _dumps(body)
        except Exception as exc:
            return 0, {"error": str(exc), "url": url}
        if self.use_requests:
            try:
                r = self.http.post(url, data=data, headers=_JSON_HEADERS, timeout=self.timeout)
            except Exception as exc:
                return 0, {"error": str(exc), "url": url}
            code, raw = r.status_code, r.content
        else:
            import http.client

            while True:
                conn, fresh = self._connect()
                try:
                    conn.request("POST", self._prefix + path, body=data, headers=_JSON_HEADERS)
                    resp = conn.getresponse()
                    code, raw = resp.status, resp.read()
                    if resp.will_close:
                        self._drop()
                    break
                except (http.client.RemoteDisconnected, BrokenPipeError, ConnectionResetError) as exc:
                    self._drop()
                    if fresh:  # a reused keep-alive socket the server closed: reconnect once
                        return 0, {"error": str(exc), "url": url}
                except Exception as exc:
                    self._drop()
                    return 0, {"error": str(exc), "url": url}
        if code == 204:
            return 204, None
        try:
            return code, json.loads(raw)
        except Exception:
            return code, raw.decode("utf-8", "replace")

    def lease(self, caps: List[str], profile: Dict[str, Any]) -> Optional[Tuple[str, List[Any]]]:
        body = {"agent": AGENT_NAME, "capabilities": {"ops": caps}, "max_tasks": MAX_TASKS,
                "timeout_ms": LEASE_TIMEOUT_MS, "labels": BASE_LABELS, "worker_profile": profile,
                "metrics": METRICS.snapshot()}
        code, resp = self.post("/v1/leases", body)
        if code == 204:
            return None
        if code == 0:
            raise RuntimeError(f"lease failed: {resp}")
        if code >= 400:
            raise RuntimeError(f"lease HTTP {code}: {resp}")
        if not isinstance(resp, dict):
            raise RuntimeError(f"lease body not dict: {resp!r}")
        lease_id, tasks = resp.get("lease_id"), resp.get("tasks")
        if not isinstance(lease_id, str) or not lease_id:
            raise RuntimeError(f"lease missing lease_id: {resp!r}")
        if not isinstance(tasks, list) or not tasks:
            return None
        return lease_id, tasks

    def result(self, lease_id: str, job_id: str, epoch: Any, status: str, result: Any, error: Any,
               attempts_done: int = 0) -> None:
        """``attempts_done``: attempts already made elsewhere (a pipelined post answered 5xx);
        at most RESULT_RETRIES + 1 attempts in all, backing off before each retry."""
        body = {"lease_id": lease_id, "job_id": job_id, "job_epoch": epoch, "status": status,
                "result": result, "error": error}
        if attempts_done > RESULT_RETRIES:
            raise RuntimeError(f"result failed after {attempts_done} attempts")
        if attempts_done:
            time.sleep(min(2.0, 0.1 * 2 ** (attempts_done - 1)))
        for attempt in range(attempts_done, RESULT_RETRIES + 1):
            code, resp = self.post("/v1/results", body)
            if 0 < code < 400:
                return
            retryable = code == 0 or code >= 500
            if not retryable or attempt == RESULT_RETRIES:
                if code == 0:
                    raise RuntimeError(f"result failed: {resp}")
                raise RuntimeError(f"result HTTP {code}: {resp}")
            time.sleep(min(2.0, 0.1 * 2**attempt))


class PipelinedPoster:
    """Result posts pipelined on ONE keep-alive connection (HTTP/1.1 request pipelining): the
    queued results go out back to back in one ``sendall`` and their responses are read in
    order afterwards, so the agent's encoding of result i+1 overlaps the controller's handling
    of result i and no post waits a round trip for the one before it. The controller still
    sees one ``POST /v1/results`` per job, in FIFO order (ref ``app.py:198-218``).

    A result whose answer is retryable (transport error, 5xx) or that the server never
    answered (it closed the connection mid-batch) is handed back to the caller, which posts
    it through the serial, retrying :meth:`Controller.result`; 4xx answers are final (logged).
    Plain ``http://`` only (``https`` controllers use the serial path)."""

    MAX_BATCH = 64

    def __init__(self, base: str, timeout: float) -> None:
        import urllib.parse

        u = urllib.parse.urlsplit(base)
        self.ok = u.scheme == "http"
        self.host, self.port = u.hostname or "localhost", u.port or 80
        self.path = (u.path.rstrip("/") + "/v1/results").encode()
        self.timeout = timeout
        self.sock = None
        self.buf = b""
        # a controller that answers HTTP/1.0 without keep-alive closes after every response:
        # pipelining cannot work against it, so it is switched off at the first sign
        self.disabled = False

    def _connect(self):
        if self.sock is None:
            self.sock = socket.create_connection((self.host, self.port), timeout=self.timeout)
            self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.buf = b""
        return self.sock

    def close(self) -> None:
        if self.sock is not None:
            try:
                self.sock.close()
            except OSError:
                pass
        self.sock, self.buf = None, b""

    def _read_until(self, sep: bytes) -> bytes:
        while sep not in self.buf:
            chunk = self.sock.recv(65536)
            if not chunk:
                raise ConnectionResetError("controller closed the connection")
            self.buf += chunk
        i = self.buf.index(sep) + len(sep)
        out, self.buf = self.buf[:i], self.buf[i:]
        return out

    def _read_n(self, n: int) -> bytes:
        while len(self.buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self.buf)))
            if not chunk:
                raise ConnectionResetError("controller closed the connection")
            self.buf += chunk
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def _response(self) -> Tuple[int, bool]:
        """(status, server will close) of the next response; its body is read and dropped.
        An HTTP/1.0 response closes unless it says ``Connection: keep-alive``."""
        head = self._read_until(b"\r\n\r\n").decode("latin-1").split("\r\n")
        status = head[0].split(" ", 2)
        code = int(status[1])
        http10 = status[0].upper() == "HTTP/1.0"
        hdr = {}
        for line in head[1:]:
            k, _, v = line.partition(":")
            hdr[k.strip().lower()] = v.strip().lower()
        if hdr.get("transfer-encoding", "") == "chunked":
            while True:
                n = int(self._read_until(b"\r\n").split(b";")[0], 16)
                self._read_n(n + 2)
                if n == 0:
                    break
        elif code != 204 and code >= 200:
            self._read_n(int(hdr.get("content-length", "0") or 0))
        conn = hdr.get("connection", "")
        return code, conn == "close" or (http10 and conn != "keep-alive")

    def post_many(self, items: List[Any]) -> List[Tuple[Any, int]]:
        """Post ``items`` ((lease_id, job_id, epoch, status, result, error) tuples) pipelined;
        returns ``(item, attempts made)`` for those that still need a (serial, retrying) post."""
        if not items:
            return []
        reqs = []
        for lease_id, job_id, epoch, status, result, error in items:
            data = _dumps({"lease_id": lease_id, "job_id": job_id, "job_epoch": epoch, "status": status,
                           "result": result, "error": error})
            reqs.append(b"POST " + self.path + b" HTTP/1.1\r\nHost: " + self.host.encode() +
                        b"\r\nContent-Type: application/json\r\nContent-Length: " + str(len(data)).encode() +
                        b"\r\n\r\n" + data)
        done = 0
        sent = False
        redo: List[Tuple[Any, int]] = []
        try:
            sock = self._connect()
            sock.sendall(b"".join(reqs))
            sent = True
            for it in items:
                code, close = self._response()
                done += 1
                if code >= 500:
                    redo.append((it, 1))
                elif code >= 400:
                    log_every("result", f"{LOG} post result error: result HTTP {code} (job {it[1]})")
                if close:
                    self.close()
                    if done < len(items):  # one response per connection: no pipelining here
                        self.disabled = True
                        log_every("result", f"{LOG} controller closes after each response; "
                                            "pipelined posts off")
                    break
        except (OSError, ValueError, IndexError) as exc:
            log_every("result", f"{LOG} pipelined post: {exc}; falling back to serial posts")
            self.close()
        # requests that went out but were never answered may have been processed: they count
        # as one attempt made (the serial path retries within RESULT_RETRIES), not as new
        return redo + [(it, 1 if sent else 0) for it in items[done:]]


class PipelinedLeaser(PipelinedPoster):
    """``POST /v1/leases`` requests pipelined on one keep-alive connection (the in-flight mode's
    feeder, :class:`LeaseFeeder`): ``n`` identical lease requests go out in one ``sendall`` and
    their answers are read in order -- each a lease (its own ``lease_id`` and tasks, exactly the
    serial loop's) or 204. The controller sees ``n`` ordinary lease requests."""

    def __init__(self, base: str, timeout: float) -> None:
        super().__init__(base, timeout)
        import urllib.parse

        u = urllib.parse.urlsplit(base)
        self.path = (u.path.rstrip("/") + "/v1/leases").encode()

    def _response_body(self) -> Tuple[int, bool, bytes]:
        head = self._read_until(b"\r\n\r\n").decode("latin-1").split("\r\n")
        status = head[0].split(" ", 2)
        code = int(status[1])
        http10 = status[0].upper() == "HTTP/1.0"
        hdr = {}
        for line in head[1:]:
            k, _, v = line.partition(":")
            hdr[k.strip().lower()] = v.strip().lower()
        body = b""
        if hdr.get("transfer-encoding", "") == "chunked":
            parts = []
            while True:
                n = int(self._read_until(b"\r\n").split(b";")[0], 16)
                parts.append(self._read_n(n + 2)[:n])
                if n == 0:
                    break
            body = b"".join(parts)
        elif code != 204 and code >= 200:
            body = self._read_n(int(hdr.get("content-length", "0") or 0))
        conn = hdr.get("connection", "")
        return code, conn == "close" or (http10 and conn != "keep-alive"), body

    def lease_many(self, n: int, body: Dict[str, Any]) -> List[Tuple[str, List[Any]]]:
        data = _dumps(body)
        req = (b"POST " + self.path + b" HTTP/1.1\r\nHost: " + self.host.encode() +
               b"\r\nContent-Type: application/json\r\nContent-Length: " + str(len(data)).encode() +
               b"\r\n\r\n" + data)
        out: List[Tuple[str, List[Any]]] = []
        n = 1 if self.disabled else n
        try:
            sock = self._connect()
            sock.sendall(req * n)
            for i in range(n):
                code, close, raw = self._response_body()
                if code == 200:
                    resp = json.loads(raw)
                    lease_id, tasks = resp.get("lease_id"), resp.get("tasks")
                    if isinstance(lease_id, str) and lease_id and isinstance(tasks, list) and tasks:
                        out.append((lease_id, tasks))
                elif code >= 400:
                    log_every("lease", f"{LOG} lease HTTP {code}: {raw[:200]!r}")
                if close:
                    self.close()
                    if i + 1 < n:
                        self.disabled = True
                    break
        except (OSError, ValueError, IndexError) as exc:
            log_every("lease", f"{LOG} pipelined lease error: {exc}")
            self.close()
        return out


class LeaseFeeder:
    """In-flight mode (``INFLIGHT_DEPTH``): a helper thread keeps up to ``depth`` leased jobs held.

    While fewer are held it sends up to ``LEASE_PIPELINE_MAX`` lease requests at once on its
    own keep-alive connection (:class:`PipelinedLeaser`); every answered lease's tasks go to
    the main loop's queue (``take``) and count as held until the main loop reports them
    finished (``done``). An idle controller (204s) gets one request per ``IDLE_SLEEP_SEC``.
    Each lease is requested with the agent's ``max_tasks`` / ``timeout_ms``: MAX_TASKS=1 (the
    reference default) means one job per lease, many leases held."""

    RATE_WINDOW_SEC = 3.0

    def __init__(self, agent: "Agent", depth: int, adaptive: bool = False) -> None:
        self.agent = agent
        self.depth = max(1, int(depth))
        # adaptive (auto depth): the sized depth until completions are measured, then the completion rate
        self.adaptive = bool(adaptive)
        self.floor = max(1, self.depth // 3)
        self._done_log: Deque[Tuple[float, int]] = deque()
        self.cv = threading.Condition()
        self.q: List[Tuple[str, List[Any]]] = []
        self.held = 0
        self.leases = 0
        self._stop = False
        self.thread = threading.Thread(target=self._loop, name="atpu-lease-feeder", daemon=True)
        self.thread.start()

    def _loop(self) -> None:
        ctl = Controller(CONTROLLER_URL, HTTP_TIMEOUT_SEC)
        pipe = PipelinedLeaser(CONTROLLER_URL, HTTP_TIMEOUT_SEC) if RESULT_PIPELINE else None
        if pipe is not None and not pipe.ok:
            pipe = None
        idle = False
        while True:
            with self.cv:
                while not self._stop and self.held >= self.limit():
                    self.cv.wait(0.2 if self.adaptive else None)
                if self._stop:
                    return
                room = self.limit() - self.held
            per = max(1, MAX_TASKS)
            n = 1 if idle else max(1, min(LEASE_PIPELINE_MAX, -(-room // per)))
            got: List[Tuple[str, List[Any]]] = []
            try:
                if pipe is not None and n > 1:
                    body = {"agent": AGENT_NAME, "capabilities": {"ops": self.agent.caps}, "max_tasks": MAX_TASKS,
                            "timeout_ms": LEASE_TIMEOUT_MS, "labels": BASE_LABELS,
                            "worker_profile": self.agent.profile, "metrics": METRICS.snapshot()}
                    got = pipe.lease_many(n, body)
                else:
                    one = ctl.lease(self.agent.caps, self.agent.profile)
                    got = [one] if one else []
            except Exception as exc:
                log_every("lease", f"{LOG} lease error: {exc}")
                time.sleep(ERROR_BACKOFF_SEC)
                continue
            if got:
                with self.cv:
                    for lease_id, tasks in got:
                        self.q.append((lease_id, tasks))
                        self.held += len(tasks)
                    self.leases += len(got)
                    self.cv.notify_all()
            idle = len(got) < n
            if not got:
                time.sleep(IDLE_SLEEP_SEC)

    def take(self, timeout: float) -> List[Tuple[str, List[Any]]]:
        with self.cv:
            if not self.q and timeout > 0:
                self.cv.wait_for(lambda: bool(self.q) or self._stop, timeout)
            out, self.q = self.q, []
            return out

    def limit(self) -> int:
        """Jobs to hold now (call with ``cv`` held): the depth, or -- adaptive -- what the jobs
        completed in the last RATE_WINDOW_SEC finish within INFLIGHT_TTL_FRACTION of the lease TTL,
        clamped to [depth / 3, depth] (the depth until a rate is measured), so held jobs do not
        outlive their leases on a slower device or model."""
        if not self.adaptive:
            return self.depth
        now = time.monotonic()
        log = self._done_log
        while log and now - log[0][0] > self.RATE_WINDOW_SEC:
            log.popleft()
        if len(log) < 2 or now - log[0][0] < 0.25:
            return self.depth
        rate = sum(n for _, n in log) / (now - log[0][0])
        cap = int(rate * LEASE_TIMEOUT_MS / 1000.0 * INFLIGHT_TTL_FRACTION)
        return max(self.floor, min(self.depth, cap))

    def done(self, n: int) -> None:
        if n:
            with self.cv:
                self.held -= n
                if self.adaptive:
                    self._done_log.append((time.monotonic(), n))
                self.cv.notify_all()

    def stop(self) -> List[Tuple[str, List[Any]]]:
        """Stop leasing; returns the leases taken but not handed to the main loop."""
        with self.cv:
            self._stop = True
            self.cv.notify_all()
        self.thread.join(timeout=HTTP_TIMEOUT_SEC + 5)
        with self.cv:
            out, self.q = self.q, []
            return out


def inflight_depth(caps: List[str], health: Optional[Dict[str, Any]]) -> int:
    """``INFLIGHT_DEPTH``: an integer, or "auto" -- on an agent with a healthy GPU and a
    batchable GPU op, the jobs the device serves within half the lease TTL at its batch sizes:
    two engine batches per batchable op (classify rows, summarize documents from worker_sizing),
    capped so that the held backlog finishes well inside LEASE_TIMEOUT_MS; 1 otherwise."""
    raw = INFLIGHT_DEPTH_RAW
    if raw not in ("", "auto"):
        try:
            return max(1, int(raw))
        except ValueError:
            return 1
    gpu_ops = set(caps) & BATCH_OPS
    if not gpu_ops or health is None or not health.get("ok", False):
        return 1
    depth = 0
    try:
        from worker_sizing import classify_batch_rows, probe_kfd

        devs = probe_kfd()
        hbm = devs[0]["total_memory_bytes"] if devs else 288 * (1 << 30)
        if gpu_ops & {"map_classify", "map_classify_tpu"}:
            depth = max(depth, 2 * classify_batch_rows(hbm, "bert-base", 128))
        if "map_summarize" in gpu_ops:
            # the concurrent searches of ATPU_INFLIGHT_PART_MAX documents each, plus the next search
            # (runtime.summarize.SummarizeStream's defaults)
            part = int(os.getenv("ATPU_INFLIGHT_PART_MAX", "256"))
            searches = int(os.getenv("ATPU_INFLIGHT_SEARCHES", "2"))
            depth = max(depth, (searches + 1) * part)
    except Exception:
        depth = 256
    # a held job must not sit out its lease TTL: cap by ~ a conservative device rate x TTL/2
    return max(1, min(depth, max(64, LEASE_TIMEOUT_MS)))


class Leaser:
    """``LEASE_PREFETCH``: lease the next task batch while the current one runs.

    The main loop leases for itself whenever nothing is ready (the reference's serial
    order, no thread hand-off for sub-millisecond jobs). A helper thread takes ONE lease
    ahead, on its own keep-alive connection (http.client is not thread-safe), only once
    the running batch has been busy for ``LEASE_PREFETCH_AFTER_MS`` (default 2 ms): GPU
    jobs then find their next lease waiting, while CPU-trivial jobs (echo) never pay for
    a second thread contending for the GIL. At most one lease is held ahead and at most
    one lease request is in flight; ``job_epoch`` and the tasks pass through untouched.
    A lease taken ahead is not started after a shutdown signal (``SHUTDOWN_AHEAD``: left to
    the lease TTL, or posted failed) and is failed with the rest on a lost DP rank.

    Controller-visible difference from the reference's serial order: a lease taken ahead
    waits for the running batch. To keep that wait short for long batches (a 1024-doc
    summarize runs ~1.5 s) the helper leases only near the batch's expected end: at
    ``max(LEASE_PREFETCH_AFTER_MS, ema - LEASE_PREFETCH_LEAD_MS)`` into the batch, ``ema``
    the moving average of recent batch durations (lead default 50 ms: several lease round
    trips), so the tasks it holds wait ~the lead, not the batch, while idle agents of the
    fleet can take the rest."""

    def __init__(self, agent: "Agent") -> None:
        self.agent = agent
        self.ctl = Controller(CONTROLLER_URL, HTTP_TIMEOUT_SEC)
        self.after = max(0.0, float(os.getenv("LEASE_PREFETCH_AFTER_MS", "2"))) / 1000.0
        self.lead = max(0.0, float(os.getenv("LEASE_PREFETCH_LEAD_MS", "50"))) / 1000.0
        self._ema: Optional[float] = None  # moving average of batch durations (s)
        self._t0 = 0.0
        self._cv = threading.Condition()
        self._ahead: Optional[Tuple[str, List[Any]]] = None
        self._inflight = False  # a lease request (either thread) is on the wire
        self._running = False   # the main loop is executing a batch
        self._epoch = 0         # batches started; one prefetch attempt per batch
        self._tried = -1
        self._stop = False
        self.thread = threading.Thread(target=self._loop, name="atpu-leaser", daemon=True)
        self.thread.start()

    # ------------------------------------------------------------- helper thread
    def _loop(self) -> None:
        with self._cv:
            while True:
                while not self._stop and not (self._running and self._ahead is None and not self._inflight
                                              and self._tried != self._epoch):
                    self._cv.wait()
                if self._stop:
                    return
                epoch = self._epoch
                # only long-running batches get a lease ahead, and only near their expected end
                delay = self.after if self._ema is None else max(self.after, self._ema - self.lead)
                self._cv.wait_for(lambda: self._stop or not self._running or self._epoch != epoch,
                                  max(0.0, self._t0 + delay - time.monotonic()))
                if self._stop:
                    return
                if not self._running or self._epoch != epoch or self._ahead is not None or self._inflight:
                    continue
                self._tried, self._inflight = epoch, True
            # lease outside the lock: the main thread keeps running its batch
                self._cv.release()
                try:
                    leased = self.ctl.lease(self.agent.caps, self.agent.profile)
                except Exception as exc:
                    log_every("lease", f"{LOG} lease error: {exc}")
                    leased = None
                finally:
                    self._cv.acquire()
                self._inflight = False
                if leased:
                    self._ahead = leased
                self._cv.notify_all()

    # --------------------------------------------------------------- main thread
    def next(self) -> Optional[Tuple[str, List[Any]]]:
        """The lease taken ahead if any, else one leased now (None on 204 / error, after
        the serial loop's IDLE_SLEEP_SEC / ERROR_BACKOFF_SEC)."""
        with self._cv:
            self._cv.wait_for(lambda: not self._inflight)
            if self._ahead is not None:
                leased, self._ahead = self._ahead, None
                return leased
            self._inflight = True
        try:
            leased = self.agent.ctl.lease(self.agent.caps, self.agent.profile)
        except Exception as exc:
            log_every("lease", f"{LOG} lease error: {exc}")
            time.sleep(ERROR_BACKOFF_SEC)
            leased = None
        else:
            if not leased:
                time.sleep(IDLE_SLEEP_SEC)
        finally:
            with self._cv:
                self._inflight = False
                self._cv.notify_all()
        return leased

    def started(self) -> None:
        with self._cv:
            self._running, self._epoch = True, self._epoch + 1
            self._t0 = time.monotonic()
            self._cv.notify_all()

    def finished(self) -> None:
        with self._cv:
            self._running = False
            dur = time.monotonic() - self._t0
            self._ema = dur if self._ema is None else 0.7 * self._ema + 0.3 * dur
            self._cv.notify_all()

    def take_ahead(self) -> Optional[Tuple[str, List[Any]]]:
        with self._cv:
            self._cv.wait_for(lambda: not self._inflight)
            leased, self._ahead = self._ahead, None
            return leased

    def pending(self) -> List[Tuple[str, List[Any]]]:
        """Leases taken from the controller but not started (rank-lost failure posts)."""
        with self._cv:
            return [self._ahead] if self._ahead is not None else []

    def stop(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self.thread.join(timeout=HTTP_TIMEOUT_SEC + 5)


_TRACE = os.getenv("MI355X_TRACE", "0").strip().lower() in ("1", "true")


def _op_span(op: str):
    """roctx range around a job under MI355X_TRACE=1 (no import cost otherwise)."""
    if not _TRACE:
        import contextlib

        return contextlib.nullcontext()
    from agent_tpu_amd.utils.trace import span

    return span(f"job:{op}")


def extract_task(task: Any) -> Tuple[str, str, Dict[str, Any], Any]:
    """-> (job_id, op, payload, job_epoch) with the reference's checks (app.py:221-234)."""
    if not isinstance(task, dict):
        raise RuntimeError(f"task not dict: {task!r}")
    job_id = task.get("id") or task.get("job_id")
    op = task.get("op")
    payload = task.get("payload") or {}
    if not isinstance(job_id, str) or not job_id:
        raise RuntimeError(f"task missing job id: {task!r}")
    if not isinstance(op, str) or not op:
        raise RuntimeError(f"task missing op: {task!r}")
    if not isinstance(payload, dict):
        raise RuntimeError(f"task payload not dict: {task!r}")
    return job_id, op, payload, task.get("job_epoch")


# ---------------------------------------------------------------- agent
class Agent:
    def __init__(self) -> None:
        from ops_loader import load_ops_lenient

        self.handlers, errors = load_ops_lenient(CAPS_LIST)
        for name, msg in errors:
            print(f"{LOG} op unavailable: {name}: {msg}", flush=True)
        # advertise only what can run: a leased-but-unloadable op would fail every job
        self.caps = [c for c in CAPS_LIST if c in self.handlers] if errors and self.handlers else list(CAPS_LIST)
        self.ctl = Controller(CONTROLLER_URL, HTTP_TIMEOUT_SEC)
        self.health = gpu_health(self.caps)
        if self.health is not None:
            print(f"{LOG} gpu health ok={self.health.get('ok')} healthy={self.health.get('healthy')} "
                  f"unhealthy={self.health.get('unhealthy', {})} {self.health.get('error', '')}", flush=True)
        self.profile = worker_profile(self.health, self.caps)
        self.exit_code = 0
        self._inflight: Dict[str, Tuple[str, Any, str]] = {}  # job_id -> (lease_id, epoch, op)
        self._inflight_lock = threading.Lock()
        # results claimed by the main loop but not yet handed to the poster (a batch's results go
        # out as ONE poster entry): kept here, under _inflight_lock, so a lost DP rank's
        # on_rank_lost still posts them before the process exits
        self._deferred: List[Any] = []
        self._deferred_lines: List[str] = []
        self._poster = None
        self._leaser: Optional[Leaser] = None
        self._feeder: Optional[LeaseFeeder] = None
        if RESULT_POST_ASYNC:
            import queue

            # bounded: backpressure on a slow controller (a whole lease of 1-row results may queue)
            self._poster = queue.Queue(maxsize=max(4, 2 * PipelinedPoster.MAX_BATCH if RESULT_PIPELINE else 4))
            threading.Thread(target=self._poster_loop, name="atpu-result-poster", daemon=True).start()

    # ---------------------------------------------------- lost-rank handling
    def _begin(self, lease_id: str, jobs: List[Tuple[str, str, Dict[str, Any], Any]]) -> None:
        with self._inflight_lock:
            for job_id, op, _, epoch in jobs:
                self._inflight[job_id] = (lease_id, epoch, op)

    def on_rank_lost(self, msg: str) -> None:
        """DP watchdog (rank 0): a rank died or hung. Fail every in-flight job naming it,
        then exit non-zero so the launcher restarts the group in fresh processes (the
        main thread may be blocked in a collective that will never complete)."""
        print(f"{LOG} {msg}; failing in-flight jobs and exiting for a restart", flush=True)
        try:
            self.flush_results()  # results of jobs that already finished go out first
        except Exception:
            pass
        with self._inflight_lock:
            jobs, self._inflight = dict(self._inflight), {}
            done, self._deferred = self._deferred, []
        pend = list(self._leaser.pending()) if self._leaser is not None else []
        if self._feeder is not None:
            with self._feeder.cv:
                pend += list(self._feeder.q)
        if pend:  # leased ahead, never started: fail them too (no TTL wait)
            for lease_id, tasks in pend:
                for task in tasks:
                    try:
                        job_id, op, _, epoch = extract_task(task)
                    except Exception:
                        continue
                    jobs.setdefault(job_id, (lease_id, epoch, op))
        err = {"type": "RankLost", "message": msg, "trace": ""}
        # this runs on the watchdog thread while the main thread may be mid-request on
        # self.ctl (one keep-alive http.client connection, not thread-safe): post on a
        # connection of its own so the failures cannot interleave with that request
        ctl = Controller(CONTROLLER_URL, HTTP_TIMEOUT_SEC)
        for item in done:  # finished before the loss: their real results
            self._post(ctl, item)
        for job_id, (lease_id, epoch, op) in jobs.items():
            try:
                ctl.result(lease_id, job_id, epoch, "failed", None, err)
            except Exception as exc:
                print(f"{LOG} post result error: {exc}", flush=True)
            log_every("exec", f"{LOG} FAIL job={job_id} op={op} err={err}")
        sys.stdout.flush()
        os._exit(EXIT_RANK_LOST)

    def run_task(self, lease_id: str, task: Any) -> None:
        try:
            job = extract_task(task)
        except Exception as exc:
            log_every("task:bad", f"{LOG} bad task: {exc} task={repr(task)[:300]}")
            return
        self._run_one(lease_id, job)

    def _run_one(self, lease_id: str, job: Tuple[str, str, Dict[str, Any], Any], defer: bool = False) -> float:
        """Run one job inline; returns its wall time (s)."""
        job_id, op, payload, epoch = job
        self._begin(lease_id, [job])
        t0 = time.time()
        out, err = None, None
        try:
            fn = self.handlers.get(op)
            if fn is None:
                raise RuntimeError(f"Unknown op '{op}'")
            with _op_span(op):
                out = fn(payload)  # inline: one job at a time per agent (ref app.py:286-287)
            if FAIL_ON_NOT_OK and isinstance(out, dict) and out.get("ok") is False:
                raise RuntimeError(str(out.get("error", "op returned ok=false")))
        except Exception as exc:
            err = {"type": type(exc).__name__, "message": str(exc), "trace": traceback.format_exc(limit=12)}
            self._note_device_fault(str(exc))
            self._note_rank_lost(exc)
        dt = time.time() - t0
        self._finish(lease_id, job_id, op, epoch, out, err, dt * 1000.0, defer)
        return dt

    def _finish(self, lease_id: str, job_id: str, op: str, epoch: Any, out: Any, err: Optional[Dict[str, Any]],
                ms: float, defer: bool = False) -> None:
        """Claim, count and post one job's result and log it (the reference's ``ok job=`` line).
        ``defer``: hold the post and the log line in the agent's deferred buffers instead (a batch
        hands its results to the poster as ONE queue entry and writes its lines in one call;
        :meth:`_flush_deferred` sends them). Claim and hold happen under one lock, so a result is
        always either in ``_inflight`` or in ``_deferred`` until it reaches the poster."""
        ok = err is None
        item = (lease_id, job_id, epoch, "succeeded" if ok else "failed", out if ok else None, None if ok else err)
        line = f"{LOG} ok job={job_id} op={op} ms={ms:.1f}" if ok else None
        with self._inflight_lock:
            if self._inflight.pop(job_id, None) is None:
                return  # already failed by the DP watchdog
            if defer:
                self._deferred.append(item)
                if line is not None:
                    self._deferred_lines.append(line)
        METRICS.job_done(ok, out)
        if not defer:
            if self._poster is not None:
                self._poster.put(item)
            else:
                self._post(self.ctl, item)
            if line is not None:
                print(line, flush=True)
        if not ok:
            log_every("exec", f"{LOG} FAIL job={job_id} op={op} ms={ms:.1f} err={err}")

    def _flush_deferred(self) -> None:
        with self._inflight_lock:
            items, self._deferred = self._deferred, []
            lines, self._deferred_lines = self._deferred_lines, []
        if items:
            if self._poster is not None:
                self._poster.put(items)  # one entry: the poster pipelines the whole batch
            else:
                for it in items:
                    self._post(self.ctl, it)
        if lines:
            sys.stdout.write("\n".join(lines) + "\n")
            sys.stdout.flush()

    @staticmethod
    def _post(ctl: "Controller", item, attempts_done: int = 0) -> None:
        try:
            ctl.result(*item, attempts_done=attempts_done)
        except Exception as exc:
            log_every("result", f"{LOG} post result error: {exc}")

    def _poster_loop(self) -> None:
        ctl = Controller(CONTROLLER_URL, HTTP_TIMEOUT_SEC)  # own keep-alive session (not shared across threads)
        pipe = PipelinedPoster(CONTROLLER_URL, HTTP_TIMEOUT_SEC) if RESULT_PIPELINE else None
        if pipe is not None and not pipe.ok:
            pipe = None
        import queue as _q

        while True:
            # queue entries: one result tuple, a list of them (a batch's results), or None (stop)
            entries = [self._poster.get()]
            if pipe is not None:  # everything already queued goes out in pipelined batches
                while entries[-1] is not None:
                    try:
                        entries.append(self._poster.get_nowait())
                    except _q.Empty:
                        break
            stop = entries[-1] is None
            batch = [it for e in entries if e is not None for it in (e if isinstance(e, list) else [e])]
            try:
                for b0 in range(0, len(batch), PipelinedPoster.MAX_BATCH):
                    part = batch[b0:b0 + PipelinedPoster.MAX_BATCH]
                    use_pipe = pipe is not None and not pipe.disabled and len(part) > 1
                    rest = pipe.post_many(part) if use_pipe else [(it, 0) for it in part]
                    for it, tried in rest:
                        self._post(ctl, it, tried)
            finally:
                for _ in entries:
                    self._poster.task_done()
            if stop:
                if pipe is not None:
                    pipe.close()
                return

    def flush_results(self) -> None:
        """Wait until every queued result is posted (shutdown / tests)."""
        if self._poster is not None:
            self._poster.join()

    def _run_batch(self, lease_id: str, jobs: List[Tuple[str, str, Dict[str, Any], Any]],
                   lease_ids: Optional[List[str]] = None) -> None:
        """Same-op jobs as ONE device batch: the jobs of one lease, or
        (in-flight mode) of several, ``lease_ids[i]`` naming job i's lease. Each job still
        gets its own result with its own lease and ``job_epoch``; a bad payload fails (or
        soft-fails) only its own result, exactly as the single-job handler would."""
        from ops import get_batch_op

        op = jobs[0][1]
        fn = get_batch_op(op)
        lids = lease_ids or [lease_id] * len(jobs)
        if lease_ids is None:
            self._begin(lease_id, jobs)
        t0 = time.time()
        try:
            with _op_span(f"{op}[x{len(jobs)}]"):
                outs = fn([p for _, _, p, _ in jobs])
            if len(outs) != len(jobs):
                raise RuntimeError(f"batch handler of {op} returned {len(outs)} results for {len(jobs)} jobs")
        except Exception as exc:  # the batch as a whole failed (e.g. a device fault): every job fails
            tr = traceback.format_exc(limit=12)
            self._note_device_fault(str(exc))
            self._note_rank_lost(exc)
            outs = [("err", exc, tr)] * len(jobs)
        ms = (time.time() - t0) * 1000.0
        for (job_id, _, _, epoch), res, lid in zip(jobs, outs, lids):
            out, err = None, None
            if res[0] == "ok":
                out = res[1]
                if FAIL_ON_NOT_OK and isinstance(out, dict) and out.get("ok") is False:
                    out, err = None, {"type": "RuntimeError", "message": str(out.get("error", "op returned ok=false")),
                                      "trace": ""}
            else:
                exc = res[1]
                tr = res[2] if len(res) > 2 else "".join(
                    traceback.format_exception(type(exc), exc, exc.__traceback__, limit=12))
                err = {"type": type(exc).__name__, "message": str(exc), "trace": tr}
            self._finish(lid, job_id, op, epoch, out, err, ms, defer=True)
        self._flush_deferred()

    def run_tasks(self, lease_id: str, tasks: List[Any]) -> None:
        """Every task of the lease, in order; with LEASE_BATCH, same-op jobs of a
        batchable op run together at the position of the first of them."""
        from ops import get_batch_op

        jobs: List[Tuple[str, str, Dict[str, Any], Any]] = []
        for task in tasks:
            try:
                jobs.append(extract_task(task))
            except Exception as exc:
                log_every("task:bad", f"{LOG} bad task: {exc} task={repr(task)[:300]}")
        groups: Dict[str, List[Tuple[str, str, Dict[str, Any], Any]]] = {}
        if LEASE_BATCH and len(jobs) > 1:
            for j in jobs:
                if j[1] in self.handlers and get_batch_op(j[1]) is not None:
                    groups.setdefault(j[1], []).append(j)
            groups = {op: js for op, js in groups.items() if len(js) > 1}
        done: set = set()
        # the results of consecutive short single jobs go to the poster (and their log lines to
        # stdout) in groups: flushed every 64 jobs, after 2 ms, before a batch, at the end of the
        # lease, and before any job that may be long -- one of another op than the job before it,
        # or after a job that itself took over DEFER_MAX_JOB_SEC -- so a finished result never
        # waits for a slow job ([echo, summarize] posts the echo first)
        n_def, t_flush, prev_op, prev_dt = 0, time.monotonic(), None, 0.0
        for j in jobs:
            op = j[1]
            if op in groups:
                self._flush_deferred()
                n_def = 0
                if op not in done:
                    done.add(op)
                    self._run_batch(lease_id, groups[op])
                prev_op = None
                continue
            if n_def and (op != prev_op or prev_dt > DEFER_MAX_JOB_SEC):
                self._flush_deferred()
                n_def, t_flush = 0, time.monotonic()
            prev_dt = self._run_one(lease_id, j, defer=True)
            prev_op = op
            n_def += 1
            if n_def >= 64 or time.monotonic() - t_flush >= 0.002:
                self._flush_deferred()
                n_def, t_flush = 0, time.monotonic()
        self._flush_deferred()

    def _note_rank_lost(self, exc: BaseException) -> None:
        """A job that lost a DP rank ends the loop after its result: exit non-zero."""
        from agent_tpu_amd.parallel.watchdog import RankLost

        global _running
        if isinstance(exc, RankLost):
            print(f"{LOG} {exc}; exiting for a restart", flush=True)
            self.exit_code = EXIT_RANK_LOST
            _running = False

    def _note_device_fault(self, msg: str) -> None:
        """A HIP fault marks the device unhealthy and re-advertises the profile.

        DP errors name global ranks (``rank K: ...``, one process per GPU, so
        rank K drives device K); a fault without a rank prefix is this
        process's own device."""
        if self.health is None:
            return
        import re

        from agent_tpu_amd.parallel.dp_ops import is_device_fault
        from agent_tpu_amd.runtime import health

        parts = re.split(r"(?:^|; )rank (\d+): ", msg)
        if len(parts) > 1:
            found = [(int(parts[i]), parts[i + 1]) for i in range(1, len(parts) - 1, 2)]
        else:
            found = [(int(os.getenv("LOCAL_RANK", "0")), msg)]
        hit = [(dev, m) for dev, m in found if is_device_fault(m)]
        for dev, m in hit:
            health.mark_unhealthy(dev, m[:200])
            print(f"{LOG} device {dev} marked unhealthy: {m[:200]}", flush=True)
        if hit:
            self.health = health.last()
            self.profile = worker_profile(self.health, self.caps)

    def loop(self) -> None:
        depth = inflight_depth(self.caps, self.health)
        if depth > 1:
            self._loop_inflight(depth)
            return
        if LEASE_PREFETCH:
            self._loop_prefetch()
            return
        while _running:
            try:
                leased = self.ctl.lease(self.caps, self.profile)
            except Exception as exc:
                log_every("lease", f"{LOG} lease error: {exc}")
                time.sleep(ERROR_BACKOFF_SEC)
                continue
            if not leased:
                time.sleep(IDLE_SLEEP_SEC)
                continue
            lease_id, tasks = leased
            self.run_tasks(lease_id, tasks)

    def _loop_prefetch(self) -> None:
        """The serial loop with the next lease taken while a batch runs (:class:`Leaser`)."""
        self._leaser = lz = Leaser(self)
        try:
            while _running:
                leased = lz.next()
                if leased is None:
                    continue
                lz.started()
                try:
                    self.run_tasks(*leased)
                finally:
                    lz.finished()
        finally:
            lz.stop()
            leased = lz.take_ahead()
            if leased is not None:
                if self.exit_code == EXIT_RANK_LOST:
                    # the DP group just lost a rank: its collectives would hang until
                    # DP_COLLECTIVE_TIMEOUT, so fail the jobs now (as on_rank_lost does)
                    self.fail_lease(*leased, {"type": "RankLost", "trace": "",
                                              "message": "DP rank lost before this lease started"})
                else:
                    # shutdown (ref app.py:239-242,257: only the in-flight work
                    # finishes): a lease taken ahead and not started is NOT run. Default: nothing
                    # is posted and the controller re-leases its tasks when the lease TTL
                    # (LEASE_TIMEOUT_MS) runs out; SHUTDOWN_AHEAD=fail posts them failed now
                    # (error type "Shutdown") for controllers that re-queue failed jobs at once.
                    self._drop_ahead(*leased)

    def _loop_inflight(self, depth: int) -> None:
        """In-flight (continuous) execution, ``INFLIGHT_DEPTH`` > 1 (see :class:`LeaseFeeder`).

        Each turn: take the jobs leased since the last turn; jobs of an op with an in-flight
        executor (``ops.register_stream_op``: map_summarize) are submitted to it and join its
        running device work at the next step boundary; jobs of a batchable op are queued and run
        as ONE batch per op (the next engine batch) together with every other job of that op
        leased meanwhile, from any number of leases; the rest run inline in arrival order. Then
        every executor advances one step and the jobs it completed are posted. A job's result is
        exactly its single-job result (ops contract); its lease and ``job_epoch`` pass through.
        Shutdown: running device work (admitted searches, the current batch) finishes; jobs
        held but not started are handled as ``SHUTDOWN_AHEAD`` says (left to the TTL or failed)."""
        from ops import get_batch_op, get_stream_op

        print(f"{LOG} in-flight mode: up to {depth} leased jobs held (MAX_TASKS={MAX_TASKS})", flush=True)
        feeder = self._feeder = LeaseFeeder(self, depth, adaptive=INFLIGHT_DEPTH_RAW in ("", "auto"))
        execs: Dict[str, Any] = {}
        ex_jobs: Dict[Tuple[str, str], Tuple[str, str, Dict[str, Any], Any]] = {}  # executor tag -> job
        held_back: List[Tuple[str, List[Any]]] = []
        try:
            while _running:
                busy = any(ex.busy() for ex in execs.values() if ex is not None)
                leases = feeder.take(0.0 if busy else 0.05)
                batches: Dict[str, List[Tuple[str, Tuple[str, str, Dict[str, Any], Any]]]] = {}
                for lease_id, tasks in leases:
                    for task in tasks:
                        try:
                            job = extract_task(task)
                        except Exception as exc:
                            log_every("task:bad", f"{LOG} bad task: {exc} task={repr(task)[:300]}")
                            feeder.done(1)
                            continue
                        op = job[1]
                        if op in self.handlers and op not in execs:
                            factory = get_stream_op(op)
                            execs[op] = factory() if factory is not None else None
                        ex = execs.get(op)
                        if ex is not None:
                            self._begin(lease_id, [job])
                            tag = (lease_id, job[0])
                            try:
                                early = ex.submit(tag, job[2])
                            except Exception as exc:
                                early = ("err", exc, traceback.format_exc(limit=12))
                            if early is not None:
                                self._finish_res(lease_id, job, early, 0.0)
                                feeder.done(1)
                            else:
                                ex_jobs[tag] = job
                        elif op in self.handlers and get_batch_op(op) is not None:
                            batches.setdefault(op, []).append((lease_id, job))
                        else:
                            self._run_one(lease_id, job, defer=True)
                            feeder.done(1)
                for op, lst in batches.items():
                    jobs = [j for _, j in lst]
                    lids = [lid for lid, _ in lst]
                    for lid, j in lst:
                        self._begin(lid, [j])
                    if len(jobs) == 1:
                        self._run_one_begun(lids[0], jobs[0])
                    else:
                        self._run_batch(lids[0], jobs, lease_ids=lids)
                    feeder.done(len(jobs))
                for op, ex in execs.items():
                    if ex is None or not ex.busy():
                        continue
                    t0 = time.time()
                    try:
                        done = ex.pump()
                    except Exception as exc:  # the executor's device work failed: its jobs fail
                        tr = traceback.format_exc(limit=12)
                        self._note_device_fault(str(exc))
                        done = [(tag, ("err", exc, tr)) for tag in ex.abort()]
                    for tag, res in done:
                        self._finish_res(tag[0], ex_jobs.pop(tag), res, (time.time() - t0) * 1000.0)
                    feeder.done(len(done))
                self._flush_deferred()
        finally:
            held_back = feeder.stop()
            # admitted device work finishes; jobs queued in an executor but not started are not run
            for op, ex in execs.items():
                if ex is None:
                    continue
                for tag in ex.cancel_queued():
                    job = ex_jobs.pop(tag)
                    with self._inflight_lock:
                        self._inflight.pop(job[0], None)
                    held_back.append((tag[0], [{"id": job[0], "op": job[1], "payload": job[2], "job_epoch": job[3]}]))
                while ex.busy():
                    for tag, res in ex.pump():
                        self._finish_res(tag[0], ex_jobs.pop(tag), res, 0.0)
            self._flush_deferred()
            for lease_id, tasks in held_back:
                self._drop_ahead(lease_id, tasks)

    def _finish_res(self, lease_id: str, job: Tuple[str, str, Dict[str, Any], Any], res: Any, ms: float) -> None:
        """Post one job's ``("ok", result) | ("err", exc[, trace])`` (batch / executor form)."""
        job_id, op, _, epoch = job
        out, err = None, None
        if res[0] == "ok":
            out = res[1]
            if FAIL_ON_NOT_OK and isinstance(out, dict) and out.get("ok") is False:
                out, err = None, {"type": "RuntimeError", "message": str(out.get("error", "op returned ok=false")),
                                  "trace": ""}
        else:
            exc = res[1]
            tr = res[2] if len(res) > 2 else "".join(traceback.format_exception(type(exc), exc, exc.__traceback__,
                                                                                  limit=12))
            err = {"type": type(exc).__name__, "message": str(exc), "trace": tr}
        self._finish(lease_id, job_id, op, epoch, out, err, ms, defer=True)

    def _run_one_begun(self, lease_id: str, job: Tuple[str, str, Dict[str, Any], Any]) -> None:
        with self._inflight_lock:
            self._inflight.pop(job[0], None)
        self._run_one(lease_id, job, defer=True)

    def _drop_ahead(self, lease_id: str, tasks: List[Any]) -> None:
        n = len(tasks)
        if SHUTDOWN_AHEAD == "fail":
            self.fail_lease(lease_id, tasks, {"type": "Shutdown", "trace": "",
                                              "message": "agent shutting down; the task was leased ahead and not started"})
            print(f"{LOG} shutdown: {n} task(s) leased ahead posted failed (lease {lease_id})", flush=True)
        else:
            print(f"{LOG} shutdown: {n} task(s) leased ahead not started; left to the lease TTL "
                  f"(lease {lease_id})", flush=True)

    def fail_lease(self, lease_id: str, tasks: List[Any], err: Dict[str, Any]) -> None:
        """Post ``failed`` for every well-formed task of a lease that will not run."""
        for task in tasks:
            try:
                job_id, op, _, epoch = extract_task(task)
            except Exception:
                continue
            self._begin(lease_id, [(job_id, op, None, epoch)])
            self._finish(lease_id, job_id, op, epoch, None, err, 0.0)


def _on_signal(signum: int, _frame: Any) -> None:
    global _running
    _running = False
    print(f"{LOG} shutdown signal {signum}", flush=True)


def main() -> int:
    global _running
    _running = True
    signal.signal(signal.SIGINT, _on_signal)
    signal.signal(signal.SIGTERM, _on_signal)
    if not CAPS_LIST:
        print(f"{LOG} no TASKS configured; exiting", flush=True)
        return 2

    world = int(os.getenv("WORLD_SIZE", "1"))
    rank = int(os.getenv("RANK", "0"))
    if world > 1:
        from agent_tpu_amd.parallel import dp_ops

        dp_ops.init_from_env()
        if rank != 0:
            return dp_ops.worker_loop()

    agent = Agent()
    if world > 1:
        from agent_tpu_amd.parallel.watchdog import Watchdog

        Watchdog(agent.on_rank_lost).start()
    print(f"{LOG} starting name={AGENT_NAME} controller={CONTROLLER_URL} ops={agent.caps}", flush=True)
    try:
        agent.loop()
    finally:
        agent.flush_results()
        if world > 1:
            from agent_tpu_amd.parallel import dp_ops, watchdog

            watchdog.stop()  # workers exiting on shutdown are not "lost"
            if agent.exit_code == 0:
                dp_ops.shutdown_workers()
    print(f"{LOG} stopped", flush=True)
    return agent.exit_code


if __name__ == "__main__":
    sys.exit(main())
