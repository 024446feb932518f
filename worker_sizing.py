"""Worker profile for the lease request, re-tuned for MI355X (288 GB HBM3E).

Schema-compatible with the reference's ``build_worker_profile()``
(``/root/reference/worker_sizing.py:221-256``): top-level ``cpu``, ``gpu``,
``tpu``, ``workers``; the CPU block keeps its formulas and env knobs
(``:44-124``). Differences:

* GPU discovery is AMD-native: the KFD topology in sysfs (no HIP context is
  created, so probing never grabs a GPU), falling back to ``amd-smi``. The
  reference only knew ``nvidia-smi`` (``:139-161``), to which MI355X is
  invisible.
* The GPU block adds HBM-derived sizing: ``hbm_gb`` per device and
  ``classify_batch_rows`` — how many BERT rows one DP rank batches, from
  (HBM − reserve − weights) / activation bytes per row, capped where the MFMA
  GEMMs are already saturated.
* ``tpu`` stays in the schema (always absent: no XLA/TPU runtime here;
  ``TPU_*`` env vars are parsed for compatibility and otherwise ignored).
* ``GPU_DISABLED`` / ``GPU_ONLY`` / ``HIP_VISIBLE_DEVICES`` /
  ``ROCR_VISIBLE_DEVICES`` replace the NVIDIA/TPU switches.
"""
from __future__ import annotations

import json
import math
import os
import subprocess
from typing import Any, Dict, List, Optional, Tuple

try:
    import psutil
except ImportError:  # pragma: no cover
    psutil = None

KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"
GIB = 1024 ** 3


# ------------------------------------------------------------------- env
def env_int(name: str, default: int) -> int:
    raw = os.getenv(name)
    try:
        return int(str(raw).strip()) if raw is not None and str(raw).strip() else default
    except ValueError:
        return default


def env_float(name: str, default: float) -> float:
    raw = os.getenv(name)
    try:
        return float(str(raw).strip()) if raw is not None and str(raw).strip() else default
    except ValueError:
        return default


def env_bool(name: str, default: bool = False) -> bool:
    raw = os.getenv(name)
    if raw is None:
        return default
    s = raw.strip().lower()
    if s in ("1", "true", "yes", "y", "on"):
        return True
    if s in ("0", "false", "no", "n", "off"):
        return False
    return default


# ------------------------------------------------------------------- cpu
def detect_cpu() -> Dict[str, Any]:
    """Same sizing model and keys as the reference CPU block."""
    total = None
    if psutil is not None:
        try:
            total = psutil.cpu_count(logical=True)
        except Exception:
            total = None
    total = int(total or os.cpu_count() or 1)
    reserved = min(env_int("CPU_RESERVED_CORES_CAP", 4), max(env_int("CPU_RESERVED_CORES_FLOOR", 1), total // 4))
    usable = max(1, total - reserved)
    factor = max(1.0, env_float("CPU_PIPELINE_FACTOR", 4.0))
    min_workers = max(1, env_int("CPU_MIN_WORKERS", 1))
    target = int(max(1, math.floor(usable * factor)))
    cap = int(max(min_workers, math.floor(usable * env_float("CPU_SOFT_CAP_MULTIPLIER", 8.0))))
    if psutil is not None:
        try:
            avail = int(getattr(psutil.virtual_memory(), "available", 0) or 0)
            per = env_int("CPU_PER_WORKER_BYTES", 32 * 1024 * 1024)
            if avail > 0 and per > 0:
                cap = max(1, min(cap, avail // per))
        except Exception:
            pass
    return {"total_cores": total, "reserved_cores": reserved, "usable_cores": usable,
            "pipeline_factor": float(factor), "target_inflight_workers": target,
            "cpu_soft_cap_workers": int(cap), "min_cpu_workers": min_workers, "max_cpu_workers": int(cap)}


# ------------------------------------------------------------------- gpu
def _read_kv(path: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    try:
        with open(path) as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 2:
                    out[parts[0]] = parts[1]
    except OSError:
        pass
    return out


def _gfx_name(version: int) -> str:
    # KFD gfx_target_version: major*10000 + minor*100 + stepping (gfx950 -> 90500)
    major, minor, step = version // 10000, (version // 100) % 100, version % 100
    return f"gfx{major}{minor:x}{step:x}"


def probe_kfd(root: Optional[str] = None) -> List[Dict[str, Any]]:
    """GPU agents from the KFD topology (CPU nodes have simd_count 0)."""
    root = root or os.getenv("ATPU_KFD_TOPOLOGY", KFD_TOPOLOGY)
    devs: List[Dict[str, Any]] = []
    try:
        nodes = sorted(os.listdir(root), key=lambda s: int(s) if s.isdigit() else 1 << 30)
    except OSError:
        return devs
    for node in nodes:
        props = _read_kv(os.path.join(root, node, "properties"))
        if int(props.get("simd_count", "0") or 0) == 0:
            continue
        mem = 0
        banks = os.path.join(root, node, "mem_banks")
        try:
            for b in os.listdir(banks):
                bp = _read_kv(os.path.join(banks, b, "properties"))
                # heap_type 1/2 = public/private frame buffer (VRAM)
                if bp.get("heap_type") in ("1", "2"):
                    mem += int(bp.get("size_in_bytes", "0") or 0)
        except OSError:
            pass
        gfx = int(props.get("gfx_target_version", "0") or 0)
        cus = int(props.get("simd_count", "0")) // max(1, int(props.get("simd_per_cu", "4") or 4))
        devs.append({"index": len(devs), "name": _gfx_name(gfx) if gfx else "amdgpu", "arch": _gfx_name(gfx),
                     "total_memory_bytes": mem, "compute_units": cus})
    return devs


DRM_ROOT = "/sys/class/drm"


def probe_gpu_busy(root: Optional[str] = None) -> List[float]:
    """Utilisation (0..1) of every AMD GPU from amdgpu's sysfs ``gpu_busy_percent``,
    in card order (no HIP context, no subprocess; the lease metric ``gpu_util``)."""
    root = root or os.getenv("ATPU_DRM_ROOT", DRM_ROOT)
    try:
        cards = [c for c in os.listdir(root) if c.startswith("card") and c[4:].isdigit()]
    except OSError:
        return []
    out: List[float] = []
    for c in sorted(cards, key=lambda c: int(c[4:])):
        dev = os.path.join(root, c, "device")
        try:
            with open(os.path.join(dev, "vendor")) as f:
                if f.read().strip().lower() != "0x1002":
                    continue
            with open(os.path.join(dev, "gpu_busy_percent")) as f:
                out.append(round(int(f.read().strip()) / 100.0, 3))
        except (OSError, ValueError):
            continue
    return out


def probe_vram(root: Optional[str] = None) -> List[Tuple[int, int]]:
    """(used, total) VRAM bytes of every AMD GPU from amdgpu's sysfs
    ``mem_info_vram_used/total``, in card order — node-wide HBM use without a HIP
    context on any device (rank 0 must not open contexts on its peers' GPUs)."""
    root = root or os.getenv("ATPU_DRM_ROOT", DRM_ROOT)
    try:
        cards = [c for c in os.listdir(root) if c.startswith("card") and c[4:].isdigit()]
    except OSError:
        return []
    out: List[Tuple[int, int]] = []
    for c in sorted(cards, key=lambda c: int(c[4:])):
        dev = os.path.join(root, c, "device")
        try:
            with open(os.path.join(dev, "vendor")) as f:
                if f.read().strip().lower() != "0x1002":
                    continue
            with open(os.path.join(dev, "mem_info_vram_used")) as f:
                used = int(f.read().strip())
            with open(os.path.join(dev, "mem_info_vram_total")) as f:
                total = int(f.read().strip())
        except (OSError, ValueError):
            continue
        out.append((used, total))
    return out


def probe_amd_smi() -> List[Dict[str, Any]]:
    try:
        out = subprocess.run(["amd-smi", "static", "--asic", "--vram", "--json"], capture_output=True, text=True,
                             timeout=20)
        data = json.loads(out.stdout) if out.returncode == 0 else None
    except Exception:
        return []
    items = data if isinstance(data, list) else (data or {}).get("gpu_data", []) if isinstance(data, dict) else []
    devs = []
    for i, g in enumerate(items):
        asic, vram = g.get("asic", {}) or {}, g.get("vram", {}) or {}
        size = vram.get("size", {})
        mib = size.get("value") if isinstance(size, dict) else size
        try:
            total = int(float(mib) * 1024 * 1024)
        except (TypeError, ValueError):
            total = 0
        devs.append({"index": i, "name": str(asic.get("market_name", "amdgpu")),
                     "arch": str(asic.get("target_graphics_version", "")), "total_memory_bytes": total,
                     "compute_units": int(asic.get("num_compute_units", 0) or 0)})
    return devs


def _visible_filter(devs: List[Dict[str, Any]]) -> Optional[List[Dict[str, Any]]]:
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        raw = os.getenv(var)
        if raw is None:
            continue
        raw = raw.strip().lower()
        if raw in ("none", "-1", "void", ""):
            return []  # set-but-empty hides every device, as in HIP/CUDA
        try:
            keep = [int(x) for x in raw.split(",") if x.strip()]
        except ValueError:
            continue
        return [dict(devs[i], index=j) for j, i in enumerate(keep) if 0 <= i < len(devs)]
    return None


def classify_batch_rows(hbm_bytes: int) -> int:
    """Rows per DP rank batch for BERT-base S=128 from the HBM budget."""
    explicit = env_int("CLASSIFY_BATCH_ROWS", 0)
    if explicit > 0:
        return explicit
    seq = env_int("CLASSIFY_SEQ_LEN", 128)
    reserve = int(env_float("HBM_RESERVE_GB", 8.0) * GIB)
    weights = 512 * 1024 * 1024  # LRU headroom for one resident BERT-large (670 MB) is budgeted below
    per_row = seq * 2 * (768 * 4 + 3 * 768 + 3072) + 2048 + 8 * seq
    fit = max(1, (hbm_bytes - reserve - 2 * weights) // per_row)
    # MFMA GEMMs saturate near M = rows*S ~ 128k tokens; bigger batches only add latency
    return int(max(64, min(fit, env_int("CLASSIFY_BATCH_ROWS_CAP", 1024))))


def detect_gpu() -> Dict[str, Any]:
    absent = {"gpu_present": False, "gpu_count": 0, "vram_gb": None, "devices": [], "max_gpu_workers": 0}
    if env_bool("GPU_DISABLED", False):
        return absent
    devs = probe_kfd() or probe_amd_smi()
    filt = _visible_filter(devs)
    if filt is not None:
        devs = filt
    if not devs:
        return absent
    biggest = max(d["total_memory_bytes"] for d in devs)
    return {
        "gpu_present": True,
        "gpu_count": len(devs),
        "vram_gb": round(biggest / GIB, 2) if biggest else None,
        "devices": devs,
        "max_gpu_workers": len(devs),  # one DP rank (process) per GPU
        "vendor": "amd",
        "hbm_gb": [round(d["total_memory_bytes"] / GIB, 2) for d in devs],
        "classify_batch_rows": classify_batch_rows(biggest) if biggest else None,
        "dp_world_size": env_int("DP_WORLD_SIZE", len(devs)),
    }


def detect_tpu() -> Dict[str, Any]:
    """Kept for schema stability; this build never claims a TPU."""
    hinted = (os.getenv("JAX_PLATFORM_NAME", "").strip().lower() == "tpu" or os.getenv("TPU_NAME") is not None
              or os.getenv("TPU_TYPE") is not None)
    if env_bool("TPU_DISABLED", False):
        hinted = False
    return {"tpu_present": False, "tpu_kind": "hinted" if hinted else None, "devices": [], "max_tpu_workers": 0}


def build_worker_profile() -> Dict[str, Any]:
    cpu, gpu, tpu = detect_cpu(), detect_gpu(), detect_tpu()
    if env_bool("GPU_ONLY", False) or env_bool("TPU_ONLY", False):
        # accelerator-only agent: the CPU only runs the agent loop and I/O
        cpu["cpu_soft_cap_workers"] = cpu["max_cpu_workers"] = cpu["min_cpu_workers"] = 1
    total = max(1, int(cpu["cpu_soft_cap_workers"]) + int(gpu.get("max_gpu_workers", 0)))
    return {"cpu": cpu, "gpu": gpu, "tpu": tpu, "workers": {"max_total_workers": total, "current_workers": 0}}


if __name__ == "__main__":
    print(json.dumps(build_worker_profile(), indent=2))
