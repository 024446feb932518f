"""In-process mock of the controller's lease/result HTTP API.

Implements ``POST /v1/leases`` and ``POST /v1/results`` exactly as the agent
uses them (ref ``/root/reference/app.py:161-218``). A scripted queue drives
the lease responses: each entry is ``(status, body)``; when the queue is empty
the controller answers 204 (idle). Result posts can be answered with injected
status codes per job id (``result_codes[job_id] = [409]`` or ``[500, 500, 200]``).
Everything the agent sends is recorded for assertions.
"""
from __future__ import annotations

import json
import threading
from collections import deque
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Deque, Dict, List, Optional, Tuple


class MockController:
    def __init__(self) -> None:
        self.leases: Deque[Tuple[int, Any]] = deque()
        self.lease_requests: List[Dict[str, Any]] = []
        self.results: List[Dict[str, Any]] = []
        self.result_codes: Dict[str, List[int]] = {}
        self.result_attempts: Dict[str, int] = {}
        # ("lease", lease_id or None) at each lease answer, ("result", job_id) when a result is
        # accepted, in order; result_delay (s) holds every result answer back (a slow controller)
        self.events: List[Tuple[str, Any]] = []
        self.result_delay = 0.0
        self.result_times: Dict[str, float] = {}  # job_id -> time.time() its result was accepted
        self.lease_times: Dict[str, float] = {}  # lease_id -> time.time() it was handed out
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)
        ctl = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            disable_nagle_algorithm = True  # headers + body are separate writes on a keep-alive socket

            def log_message(self, *_a):  # quiet
                pass

            def _send(self, code: int, body: Any = None) -> None:
                data = b"" if body is None else (body if isinstance(body, bytes) else json.dumps(body).encode())
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                if data:
                    self.wfile.write(data)

            def do_POST(self):  # noqa: N802
                n = int(self.headers.get("Content-Length", "0"))
                body = json.loads(self.rfile.read(n) or b"{}")
                if self.path == "/v1/leases":
                    with ctl._cv:
                        ctl.lease_requests.append(body)
                        item = ctl.leases.popleft() if ctl.leases else (204, None)
                        lid = item[1].get("lease_id") if isinstance(item[1], dict) else None
                        ctl.events.append(("lease", lid))
                        if lid:
                            import time as _t

                            ctl.lease_times[lid] = _t.time()
                        ctl._cv.notify_all()
                    self._send(*item)
                elif self.path == "/v1/results":
                    jid = body.get("job_id")
                    if ctl.result_delay:
                        import time

                        time.sleep(ctl.result_delay)
                    with ctl._cv:
                        ctl.result_attempts[jid] = ctl.result_attempts.get(jid, 0) + 1
                        codes = ctl.result_codes.get(jid)
                        code = codes.pop(0) if codes else 200
                        if code < 400:
                            import time as _t

                            ctl.result_times[jid] = _t.time()
                            ctl.results.append(body)
                            ctl.events.append(("result", jid))
                        ctl._cv.notify_all()
                    self._send(code, {"ok": code < 400})
                else:
                    self._send(404, {"error": "not found"})

        self.server = ThreadingHTTPServer(("127.0.0.1", 0), Handler)
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.server.server_address[1]}"

    def start(self) -> "MockController":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.server.shutdown()
        self.server.server_close()

    def lease(self, *tasks: Any, lease_id: str = "L1", status: int = 200, body: Optional[Any] = None) -> None:
        with self._lock:
            self.leases.append((status, body if body is not None else {"lease_id": lease_id, "tasks": list(tasks)}))

    def wait(self, pred, timeout: float = 60.0) -> bool:
        with self._cv:
            return self._cv.wait_for(lambda: pred(self), timeout=timeout)
