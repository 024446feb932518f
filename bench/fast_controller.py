"""A faster stand-in for ``tests/integration/mock_controller.MockController`` in benchmarks.

The test mock is a ``ThreadingHTTPServer``: ~150-250 us of Python per request in the bench
process, so at hundreds of 1-row jobs per lease it, not the agent, set the jobs/s ceiling
(~6-7k results/s). This one is an asyncio server on one event-loop thread with a minimal
HTTP/1.1 parser (keep-alive, pipelined requests answered in order, Content-Length bodies),
pre-encoded answers, and result bodies kept as raw bytes until read. Same surface as the
benches use: ``lease(*tasks, lease_id=)``, ``wait(pred, timeout)``, ``results``,
``lease_requests``, ``url``, ``start()`` / ``stop()``. Wire protocol: ref ``app.py:161-218``.
"""
from __future__ import annotations

import asyncio
import json
import threading
import time
from collections import deque
from typing import Any, Deque, Dict, List

_OK = b'{"ok":true}'


def _answer(code: int, body: bytes = b"") -> bytes:
    reason = {200: b"OK", 204: b"No Content", 404: b"Not Found"}.get(code, b"X")
    return (b"HTTP/1.1 " + str(code).encode() + b" " + reason + b"\r\nContent-Type: application/json\r\n"
            b"Content-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body)


_RESULT_OK = _answer(200, _OK)
_IDLE = _answer(204)


class FastController:
    def __init__(self) -> None:
        self.leases: Deque[bytes] = deque()
        self._raw_leases: List[bytes] = []
        self._raw_results: List[bytes] = []
        self.result_t: List[float] = []  # perf_counter() of each result, in arrival order
        self.lease_t: List[float] = []   # perf_counter() of each answered (non-idle) lease, in order
        self._results: List[Dict[str, Any]] = []
        self._lease_reqs: List[Dict[str, Any]] = []
        self._cv = threading.Condition()
        self._loop = None
        self._server = None
        self._thread = None
        self.url = ""

    # ------------------------------------------------------------------ scripting
    def lease(self, *tasks: Dict[str, Any], lease_id: str = "") -> None:
        lid = lease_id or f"L{len(self.leases) + len(self._raw_leases) + 1}"
        body = json.dumps({"lease_id": lid, "tasks": list(tasks)}, separators=(",", ":")).encode()
        with self._cv:
            self.leases.append(_answer(200, body))

    @property
    def results(self) -> List[Dict[str, Any]]:
        with self._cv:
            raw = self._raw_results[len(self._results):]
        self._results.extend(json.loads(b) for b in raw)
        return self._results

    @property
    def lease_requests(self) -> List[Dict[str, Any]]:
        with self._cv:
            raw = self._raw_leases[len(self._lease_reqs):]
        self._lease_reqs.extend(json.loads(b) for b in raw)
        return self._lease_reqs

    def n_results(self) -> int:
        with self._cv:
            return len(self._raw_results)

    def wait(self, pred, timeout: float) -> bool:
        """``pred(self)`` polled until true; ``n_results()`` is the cheap progress probe."""
        end = time.time() + timeout
        while time.time() < end:
            if pred(self):
                return True
            time.sleep(0.002)
        return bool(pred(self))

    # ------------------------------------------------------------------ server
    async def _conn(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            while True:
                head = await reader.readuntil(b"\r\n\r\n")
                line, _, rest = head.partition(b"\r\n")
                n = 0
                for h in rest.split(b"\r\n"):
                    if h[:15].lower() == b"content-length:":
                        n = int(h[15:])
                body = await reader.readexactly(n) if n else b""
                path = line.split(b" ", 2)[1]
                if path.endswith(b"/v1/results"):
                    with self._cv:
                        self._raw_results.append(body)
                        self.result_t.append(time.perf_counter())
                    writer.write(_RESULT_OK)
                elif path.endswith(b"/v1/leases"):
                    with self._cv:
                        self._raw_leases.append(body)
                        out = self.leases.popleft() if self.leases else _IDLE
                        if out is not _IDLE:
                            self.lease_t.append(time.perf_counter())
                    writer.write(out)
                else:
                    writer.write(_answer(404, b'{"error":"not found"}'))
                if not reader._buffer:  # pipelined requests waiting: answer them first, flush once
                    await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionResetError, BrokenPipeError):
            pass
        finally:
            writer.close()

    def start(self) -> "FastController":
        ready = threading.Event()

        def run():
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            self._server = self._loop.run_until_complete(asyncio.start_server(self._conn, "127.0.0.1", 0))
            self.url = f"http://127.0.0.1:{self._server.sockets[0].getsockname()[1]}"
            ready.set()
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()
        ready.wait(10)
        return self

    def stop(self) -> None:
        if self._loop is not None:
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(timeout=5)
