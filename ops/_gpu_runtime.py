"""Device-resident model cache for accelerator ops.

MI355X counterpart of ``/root/reference/ops/_tpu_runtime.py``:

* :func:`get_model_path` keeps the reference's precedence (payload value, then
  env, then a default; ref ``:23-31``) with ``GPU_MODEL_PATH`` /
  ``CLASSIFY_MODEL`` in place of ``TPU_MODEL_PATH``.
* :func:`get_gpu_handle` replaces the single-slot, unlocked interpreter cache
  (ref ``:9-12,39-61``; switching models rebuilt it every time, SURVEY.md
  §2.4.13) with a mutex-guarded LRU of engines resident in HBM.

A "model path" is a BERT preset (``bert-base``, ``bert-large``, ``bert-tiny``),
optionally with query options ``bert-base?labels=5&seed=3&batch=512``, or a
``.safetensors`` file whose config sits next to it as ``<file>.json``.
Random-init weights are seeded, so every rank/host builds identical weights;
under DP rank 0 initialises and broadcasts them (RCCL).
"""
from __future__ import annotations

import json
import os
import threading
from collections import OrderedDict
from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple
from urllib.parse import parse_qs, urlsplit

DEFAULT_MODEL = "bert-base"


def get_model_path(requested: Optional[str] = None) -> str:
    return requested or os.environ.get("GPU_MODEL_PATH") or os.environ.get("CLASSIFY_MODEL") or DEFAULT_MODEL


@dataclass(frozen=True)
class ModelSpec:
    path: str
    preset: str
    labels: int
    seed: int
    batch_rows: int
    seq_len: int
    file: Optional[str] = None


def parse_spec(path: str) -> ModelSpec:
    from agent_tpu_amd.models.bert import PRESETS

    u = urlsplit(path)
    q = {k: v[-1] for k, v in parse_qs(u.query).items()}
    base = u.path if u.scheme in ("", "file") else path
    seq = int(q.get("seq", os.getenv("CLASSIFY_SEQ_LEN", "128")))
    batch = int(q.get("batch", os.getenv("CLASSIFY_BATCH_ROWS", "0")) or 0)
    if base in PRESETS:
        return ModelSpec(path, base, int(q.get("labels", os.getenv("CLASSIFY_NUM_LABELS", "2"))),
                         int(q.get("seed", os.getenv("MODEL_SEED", "0"))), batch, seq)
    if base.endswith(".safetensors"):
        if not os.path.exists(base):
            raise FileNotFoundError(f"GPU model not found: {base}")
        with open(base + ".json") as f:
            meta = json.load(f)
        return ModelSpec(path, meta.get("preset", DEFAULT_MODEL), int(meta.get("num_labels", 2)), 0, batch, seq,
                         file=base)
    raise FileNotFoundError(f"GPU model not found: {path}")


class GpuHandle:
    """A loaded model: config + device engine."""

    def __init__(self, spec: ModelSpec, cfg, engine):
        self.spec = spec
        self.model_path = spec.path
        self.cfg = cfg
        self.engine = engine
        self.load_ms: Dict[str, Any] = {}  # cold-load phases (set by _build_handle)
        self.fresh = True  # built by this call (the first job reports load_ms as its cold load)


def _load_host_pack(spec: ModelSpec, cfg):
    from agent_tpu_amd.models.bert import init_random

    if spec.file:
        from safetensors.torch import load_file

        from agent_tpu_amd.models.bert import param_specs
        from agent_tpu_amd.models.params import ParamPack

        pack = ParamPack(param_specs(cfg))
        tensors = load_file(spec.file)
        missing = [n for n in pack.names() if n not in tensors]
        if missing:
            raise KeyError(f"{spec.file}: missing tensors {missing[:4]}{' ...' if len(missing) > 4 else ''}")
        for name in pack.names():
            pack[name].copy_(tensors[name])
        return pack
    return init_random(cfg, seed=spec.seed)


def _build_handle(model_path: str, device) -> GpuHandle:
    """Load a model on this rank, or on every rank of the DP group together.

    Random-init specs are built on the device by every rank (``params.rand_fill``: the
    same bits everywhere, no host init, no H2D copy, no broadcast). A ``.safetensors``
    spec follows ``dp_ops.load_collectively``: rank 0 loads it on the host and copies it
    to its GPU, the other ranks allocate the destination, errors are exchanged, and only
    then does the C1 broadcast run (all ranks or none); the engine build is exchanged
    again. ``handle.load_ms`` records the phases (weights, engine).
    """
    from agent_tpu_amd.models.bert import config_for, param_specs
    from agent_tpu_amd.models.params import ParamPack
    from agent_tpu_amd.parallel.dp import broadcast_pack, is_dist, world
    from agent_tpu_amd.parallel.dp_ops import load_collectively
    from agent_tpu_amd.runtime.classify import ClassifyEngine

    import time

    from agent_tpu_amd.models.bert import init_random

    dist_on = is_dist()
    box = {"t0": time.perf_counter()}

    def sync():
        if getattr(device, "type", "cpu") == "cuda":
            import torch

            torch.cuda.synchronize(device)

    def local():
        spec = parse_spec(model_path)
        cfg = config_for(spec.preset, num_labels=spec.labels)
        box.update(spec=spec, cfg=cfg)
        if not spec.file:
            return init_random(cfg, seed=spec.seed, device=device)
        if dist_on and world()[0] != 0:
            return ParamPack(param_specs(cfg), device=device)
        return _load_host_pack(spec, cfg).to(device)

    def collective(pack):
        out = broadcast_pack(pack, box["cfg"], device) if dist_on and box["spec"].file else pack
        sync()
        box["t1"] = time.perf_counter()
        return out

    def post(pack):
        spec, cfg = box["spec"], box["cfg"]
        batch = spec.batch_rows or _auto_batch_rows(spec.preset, spec.seq_len)
        eng = ClassifyEngine(cfg, pack, device, batch_rows=batch, seq_len=spec.seq_len,
                             topk=min(cfg.num_labels, 64))
        sync()
        h = GpuHandle(spec, cfg, eng)
        t2 = time.perf_counter()
        h.load_ms = {"weights_ms": (box["t1"] - box["t0"]) * 1e3, "engine_ms": (t2 - box["t1"]) * 1e3,
                     "total_ms": (t2 - box["t0"]) * 1e3, "source": "file" if spec.file else "device_rand"}
        return h

    return load_collectively(local, collective, post)


def _auto_batch_rows(preset: str = "bert-base", seq_len: int = 128) -> int:
    """The engine batch of a served model: the SAME function the worker profile advertises
    (``worker_sizing.classify_batch_rows``, per model and sequence length)."""
    from worker_sizing import classify_batch_rows

    try:
        import torch

        total = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory
    except Exception:
        total = 288 * 1024 ** 3
    return classify_batch_rows(total, preset, seq_len)


_lock = threading.Lock()
_cache: "OrderedDict[Tuple[str, str], GpuHandle]" = OrderedDict()


def lru_capacity() -> int:
    return max(1, int(os.getenv("MODEL_LRU_SIZE", "4")))


def lru_budget_bytes(device) -> int:
    """HBM budget for resident models: ``MODEL_LRU_GB`` or
    25 % of the device's memory. Eviction is LRU and deterministic, so every DP
    rank (same request sequence, same configs) evicts the same models."""
    gb = os.getenv("MODEL_LRU_GB", "").strip()
    if gb:
        return int(float(gb) * 2**30)
    try:
        import torch

        return int(torch.cuda.get_device_properties(device).total_memory * 0.25)
    except Exception:
        return 64 * 2**30


def device_for_rank():
    import torch

    if os.getenv("CLASSIFY_DEVICE", "").strip().lower() == "cpu":
        return torch.device("cpu")  # fp32 PyTorch oracle path (CPU tests of the op forms)
    if not torch.cuda.is_available():
        raise RuntimeError("No ROCm GPU available (torch.cuda.is_available() is False)")
    # modulo: ranks may share a device in single-GPU rehearsals (gloo backend)
    local = int(os.getenv("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    return torch.device("cuda", local)


def get_gpu_handle(model_path: str, device=None) -> GpuHandle:
    """Cached handle for ``model_path``.

    Under a DP process group this is a collective: call it only from a
    dispatched DP task body (``dp_ops.dispatch``), where every rank asks for
    the same models in the same order. The caches of all ranks then hold the
    same keys, so they agree on hit or miss, and a miss broadcasts the
    weights from rank 0 (C1) with every rank taking part.
    """
    from agent_tpu_amd.parallel.dp import is_dist
    from agent_tpu_amd.parallel.dp_ops import in_task

    if is_dist() and not in_task():
        raise RuntimeError("get_gpu_handle under a DP process group must run inside a dispatched DP task "
                           "(dp_ops.dispatch), so that every rank loads the model together")
    device = device if device is not None else device_for_rank()
    key = (model_path, str(device))
    with _lock:
        h = _cache.get(key)
        if h is not None:
            _cache.move_to_end(key)
            return h
        h = _build_handle(model_path, device)
        _cache[key] = h
        budget = lru_budget_bytes(device)
        evicted = False
        while len(_cache) > 1 and (len(_cache) > lru_capacity() or _resident_bytes() > budget):
            _cache.popitem(last=False)
            evicted = True
        if evicted:
            import torch

            torch.cuda.empty_cache()  # hand the evicted packs/graph pools back to the device
        return h


def _resident_bytes() -> int:
    return sum(h.engine.memory_bytes() for h in _cache.values())


def cache_info() -> Dict[str, Any]:
    with _lock:
        return {"entries": [k[0] for k in _cache], "capacity": lru_capacity(), "resident_bytes": _resident_bytes()}
