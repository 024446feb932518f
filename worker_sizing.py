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


# Served model shapes (kept in step with the presets in agent_tpu_amd/models/{bert,t5,bart}.py by
# tests/contract/test_worker_sizing.py; this module stays importable without torch, like the reference's).
#   classify: hidden, intermediate, layers, vocab, max_positions
CLASSIFY_DIMS = {"bert-base": (768, 3072, 12, 30522, 512), "bert-large": (1024, 4096, 24, 30522, 512),
                 "bert-tiny": (256, 1024, 2, 4096, 512)}
#   summarize: d_model, d_ff, enc_layers, dec_layers, vocab
SUMMARIZE_DIMS = {"t5-base": (768, 3072, 12, 12, 32128), "t5-small": (512, 2048, 6, 6, 32128),
                  "bart-large-cnn": (1024, 4096, 12, 12, 50264), "bart-large": (1024, 4096, 12, 12, 50264),
                  "bart-base": (768, 3072, 6, 6, 50264)}
CLASSIFY_TOKENS_PER_BATCH = 131072  # M = rows*S where the MFMA GEMMs saturate (docs/PERF_NOTES.md, Batch size)
CLASSIFY_MAX_ROW_BYTES = 2048       # agent_tpu_amd.tokenizer.DEFAULT_MAX_ROW_BYTES (device text staging)
SUMMARIZE_DOCS_TARGET = 1024        # docs/PERF_NOTES.md: 1024 docs/step is the T5 / BART throughput plateau
SUMMARIZE_SRC, SUMMARIZE_BEAMS, SUMMARIZE_MAX_LEN = 1024, 4, 130  # ref ops/map_summarize.py:49,53-59


def _activation_budget(hbm_bytes: int) -> int:
    """HBM one engine may spend on activations: what is left after HBM_RESERVE_GB and the
    model LRU's share (MODEL_LRU_GB, default 25 % of the device: ops/_gpu_runtime.lru_budget_bytes)."""
    reserve = int(env_float("HBM_RESERVE_GB", 8.0) * GIB)
    lru_gb = env_float("MODEL_LRU_GB", 0.0)
    lru = int(lru_gb * GIB) if lru_gb > 0 else hbm_bytes // 4
    return max(0, hbm_bytes - reserve - lru)


def classify_row_bytes(model: str = "bert-base", seq_len: int = 128, slots: int = 2) -> int:
    """Device bytes one batch row costs the ClassifyEngine (agent_tpu_amd/runtime/classify.py):
    per staging slot (``slots`` batches in flight, each with its own graph pool) the text
    staging, ids/lengths and the LayerNorm-folded encoder's live activations (bf16): the
    layer input, the attention context (the fused QKV + attention kernel never writes the
    [S, 3H] QKV), the out-proj sum, the FFN intermediate and the FFN2 sum, plus per-row
    LayerNorm statistics (fp32 partials of up to 4 column tiles and the finalized pair)."""
    H, I, _, _, _ = CLASSIFY_DIMS[model]
    S = int(seq_len)
    act = S * 2 * (4 * H + I) + S * 4 * (2 * 4 + 2)
    return slots * (CLASSIFY_MAX_ROW_BYTES + 4 + S * 4 + 4 + act)


def classify_batch_rows(hbm_bytes: int, model: str = "bert-base", seq_len: Optional[int] = None,
                        slots: int = 2) -> int:
    """Rows per DP-rank batch for the served classify model: the GEMM-saturating token count
    (``CLASSIFY_TOKENS_PER_BATCH`` / S) unless the HBM activation budget is smaller.
    ``CLASSIFY_BATCH_ROWS`` overrides; ``CLASSIFY_BATCH_ROWS_CAP`` caps."""
    explicit = env_int("CLASSIFY_BATCH_ROWS", 0)
    if explicit > 0:
        return explicit
    if model not in CLASSIFY_DIMS:
        model = "bert-base"
    seq = int(seq_len) if seq_len else env_int("CLASSIFY_SEQ_LEN", 128)
    fit = _activation_budget(hbm_bytes) // classify_row_bytes(model, seq, slots)
    target = max(64, CLASSIFY_TOKENS_PER_BATCH // max(1, seq))
    rows = min(fit, target, env_int("CLASSIFY_BATCH_ROWS_CAP", 1 << 30))
    if rows >= 64:
        rows -= rows % 64  # whole 2-row x 128-token GEMM tiles
    return int(max(1, rows))


def summarize_doc_bytes(model: str = "t5-base", src: int = SUMMARIZE_SRC, beams: int = SUMMARIZE_BEAMS,
                        max_len: int = SUMMARIZE_MAX_LEN) -> int:
    """Device bytes per document of a beam search (agent_tpu_amd/runtime/summarize.py):
    the encoder's cross K/V for every decoder layer (one copy per document), the
    self-attention KV cache of every beam up to ``max_len``, the encoder activations at
    ``src`` tokens, and the per-beam decode state (hidden rows, token history, LM-head
    partials of the fused top-k: per 128-token vocabulary tile a max, a sum and 16
    candidates)."""
    return summarize_doc_bytes_dims(SUMMARIZE_DIMS[model], src, beams, max_len)


def summarize_doc_bytes_dims(dims: Tuple[int, int, int, int, int], src: int = SUMMARIZE_SRC,
                             beams: int = SUMMARIZE_BEAMS, max_len: int = SUMMARIZE_MAX_LEN) -> int:
    """:func:`summarize_doc_bytes` for explicit (d_model, d_ff, enc_layers, dec_layers, vocab)."""
    d, f, _, dec, V = dims
    cross = dec * 2 * src * d * 2
    self_kv = beams * dec * 2 * max_len * d * 2
    enc_act = src * 2 * (2 * d + 3 * d + d + f)
    step = beams * (6 * d * 2 + max_len * 4 + ((V + 127) // 128) * (2 + 16 * 2) * 4)
    return cross + self_kv + enc_act + step


def summarize_batch_docs(hbm_bytes: int, model: Any = "t5-base", src: int = SUMMARIZE_SRC) -> int:
    """Documents per device batch (``model``: a SUMMARIZE_DIMS name or a dims tuple): the
    throughput plateau unless HBM is smaller. ``SUMMARIZE_BATCH_DOCS`` overrides.
    SummarizeEngine.run splits a larger call into batches of this size."""
    explicit = env_int("SUMMARIZE_BATCH_DOCS", 0)
    if explicit > 0:
        return explicit
    dims = model if isinstance(model, tuple) else SUMMARIZE_DIMS.get(model, SUMMARIZE_DIMS["t5-base"])
    fit = _activation_budget(hbm_bytes) // summarize_doc_bytes_dims(dims, src)
    return int(max(1, min(fit, SUMMARIZE_DOCS_TARGET)))


RISK_RECORD_BYTES = 24  # slot bytes per record of a streamed risk chunk (agent_tpu_amd/runtime/risk.py)


def risk_chunk_rows(hbm_bytes: int) -> int:
    """Records per streamed chunk of a risk_accumulate CSV shard (agent_tpu_amd/runtime/risk.py):
    two pinned host slots and two device slots, each holding a chunk's raw record bytes
    (``RISK_RECORD_BYTES`` per record, byte-limited chunks for longer records) and its 4-B record
    offsets. The host staging (``RISK_STAGING_MB``, default 256 MiB for both slots) bounds it, so
    the agent's memory does not grow with ``shard_size``; ``RISK_CHUNK_ROWS`` overrides."""
    explicit = env_int("RISK_CHUNK_ROWS", 0)
    if explicit > 0:
        return explicit
    per = 2 * (RISK_RECORD_BYTES + 4)
    host = env_int("RISK_STAGING_MB", 256) * (1 << 20) // per
    dev = max(1, _activation_budget(hbm_bytes) // per) if hbm_bytes else host
    return int(max(1 << 16, min(host, dev)))


def gpu_capacity(hbm_bytes: int) -> Dict[str, Any]:
    """What this device can take per batch, for every servable model: advertised in the
    lease's worker profile so a controller can size leases (ref worker_sizing.py:221-256
    advertised only worker counts)."""
    seq = env_int("CLASSIFY_SEQ_LEN", 128)
    return {
        "classify_seq_len": seq,
        "classify_batch_rows": {m: classify_batch_rows(hbm_bytes, m, seq) for m in CLASSIFY_DIMS if m != "bert-tiny"},
        "summarize_source_tokens": SUMMARIZE_SRC,
        "summarize_beams": SUMMARIZE_BEAMS,
        "summarize_batch_docs": {m: summarize_batch_docs(hbm_bytes, m) for m in ("t5-base", "bart-large-cnn")},
        "risk_chunk_rows": risk_chunk_rows(hbm_bytes),
    }


def _served_classify_model() -> str:
    """Preset of the default classify model (GPU_MODEL_PATH / CLASSIFY_MODEL, ops/_gpu_runtime.py)."""
    raw = os.getenv("GPU_MODEL_PATH") or os.getenv("CLASSIFY_MODEL") or "bert-base"
    name = raw.split("?", 1)[0].strip()
    return name if name in CLASSIFY_DIMS else "bert-base"


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
        "classify_batch_rows": classify_batch_rows(biggest, _served_classify_model()) if biggest else None,
        "capacity": gpu_capacity(biggest) if biggest else None,
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
