"""GPU health check at agent start-up and after device faults.

``check()`` enumerates the devices through the native HIP query (arch, CUs,
clock, HBM total/free), requires gfx950, and runs a tiny MFMA GEMM probe on
each device against a torch fp32 reference. The result is advertised in the
worker profile (``gpu.health``) and failed devices are listed as unhealthy so
the controller sees the reduced capacity; ``mark_unhealthy`` records a device
that faulted during a job (per-rank errors already carry the rank id).
"""
from __future__ import annotations

import threading
from typing import Any, Dict, List, Optional

EXPECTED_ARCH = "gfx950"
_lock = threading.Lock()
_unhealthy: Dict[int, str] = {}
_last: Optional[Dict[str, Any]] = None


def _probe(index: int) -> Optional[str]:
    """Return an error string, or None when the MFMA GEMM probe matches torch."""
    import torch

    from .. import ops

    try:
        dev = torch.device("cuda", index)
        g = torch.Generator().manual_seed(index)
        a = torch.randn(64, 128, generator=g).to(torch.bfloat16)
        w = torch.randn(256, 128, generator=g).to(torch.bfloat16)
        # the kernel launches on the CURRENT device's stream: make device ``index`` current
        with torch.cuda.device(dev):
            y = ops.linear(a.to(dev), w.to(dev)).float().cpu()
        ref = a.float() @ w.float().t()
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        if not err < 2e-2:
            return f"GEMM probe mismatch (rel err {err:.3g})"
        return None
    except Exception as exc:  # a dead/faulted device raises here
        return f"{type(exc).__name__}: {exc}"


def check(probe: bool = True, only: Optional[List[int]] = None) -> Dict[str, Any]:
    """``{ok, devices:[...], healthy:[idx], unhealthy:{idx: reason}}``; never raises.

    ``only``: the device indices this process may touch (MFMA probe, free-HBM
    query). A DP rank passes its own device so it never creates a HIP context on
    a peer's GPU; :func:`check_dp` gathers the ranks' answers. ``None`` = all."""
    global _last
    out: Dict[str, Any] = {"ok": False, "devices": [], "healthy": [], "unhealthy": {}}
    try:
        import torch

        if not torch.cuda.is_available():
            out["error"] = "no ROCm device visible"
            _last = out
            return out
        from .._native import native

        mem_of = only[0] if only else -1
        devs = native().device_query(mem_of)
    except Exception as exc:
        out["error"] = f"{type(exc).__name__}: {exc}"
        _last = out
        return out
    for d in devs:
        idx = int(d["index"])
        if only is not None and idx not in only:
            continue
        info = {k: d[k] for k in ("index", "name", "arch", "compute_units", "clock_khz")}
        info["hbm_total_gb"] = round(d["total_memory_bytes"] / 2**30, 2)
        if d.get("free_memory_known", True):
            info["hbm_free_gb"] = round(d["free_memory_bytes"] / 2**30, 2)
        out["devices"].append(info)
        reason = None
        if not str(d["arch"]).startswith(EXPECTED_ARCH):
            reason = f"arch {d['arch']} is not {EXPECTED_ARCH}"
        elif probe:
            reason = _probe(idx)
        with _lock:
            reason = reason or _unhealthy.get(idx)
        if reason:
            out["unhealthy"][idx] = reason
        else:
            out["healthy"].append(idx)
    out["ok"] = bool(out["healthy"])
    _last = out
    return out


def merge(parts: List[Dict[str, Any]]) -> Dict[str, Any]:
    """One node view from per-rank :func:`check` results (each covering its own device)."""
    out: Dict[str, Any] = {"ok": False, "devices": [], "healthy": [], "unhealthy": {}}
    errs = []
    for p in parts:
        out["devices"] += p.get("devices", [])
        out["healthy"] += p.get("healthy", [])
        out["unhealthy"].update(p.get("unhealthy", {}))
        if p.get("error"):
            errs.append(p["error"])
    ranks = [p["rank_info"] for p in parts if p.get("rank_info")]
    if ranks:
        out["ranks"] = sorted(ranks, key=lambda r: r["rank"])
    out["devices"].sort(key=lambda d: d["index"])
    out["healthy"] = sorted(set(out["healthy"]) - set(out["unhealthy"]))
    out["ok"] = bool(out["healthy"])
    if errs:
        out["error"] = "; ".join(errs)
    return out


def set_last(res: Dict[str, Any]) -> Dict[str, Any]:
    global _last
    with _lock:
        for idx, reason in _unhealthy.items():
            res["unhealthy"].setdefault(idx, reason)
            if idx in res["healthy"]:
                res["healthy"].remove(idx)
        res["ok"] = bool(res["healthy"])
        _last = res
    return res


def mark_unhealthy(index: int, reason: str) -> None:
    with _lock:
        _unhealthy[int(index)] = reason
        if _last is not None:
            _last["unhealthy"][int(index)] = reason
            if int(index) in _last["healthy"]:
                _last["healthy"].remove(int(index))
            _last["ok"] = bool(_last["healthy"])


def last() -> Optional[Dict[str, Any]]:
    return _last


def healthy_count() -> Optional[int]:
    return None if _last is None else len(_last["healthy"])
