"""Per-rank host placement: CPU affinity and host thread budgets by the GPU's NUMA node.

One process per GPU (ref ``app.py:286-287`` runs one inline worker). On a
two-socket MI355X node the 8 GPUs hang off two NUMA nodes, and every rank's host work --
the CSV stager threads and pinned double buffer of ``classify_table``, the risk stream's
copy threads, torch's intra-op pool -- belongs on the cores of ITS GPU's node, split with
the other ranks of that node rather than each rank sizing its pools for the whole machine
(8 ranks x ``min(16, cpu_count)`` risk threads was 128 threads on one node).

:func:`place_rank` runs in every rank at import (``launch.ensure_rank_env``), before
anything touches the GPU (no HIP call: the GPU -> NUMA map comes from sysfs):

* GPU -> NUMA node: the KFD topology (``/sys/class/kfd/kfd/topology/nodes``): a GPU
  node's io_link to a CPU node (CPU nodes are the NUMA nodes, in order); fallback the PCI
  device's ``numa_node`` under ``/sys/class/drm``;
* NUMA node -> cores: ``/sys/devices/system/node/node<N>/cpulist`` intersected with the
  process's allowed set;
* the ranks of this node whose GPUs share a NUMA node split its cores into contiguous,
  disjoint chunks (rank order); a node with no usable cores falls back to an even split
  of the allowed set over all local ranks;
* ``sched_setaffinity`` to the chunk, and the chunk's size becomes the host thread budget
  (:func:`host_threads`, ``OMP_NUM_THREADS`` / ``ATPU_HOST_THREADS`` defaults,
  ``torch.set_num_threads`` when torch is loaded).

Applied when several ranks share the node (``LOCAL_WORLD_SIZE`` > 1, both launch forms:
an external ``torch.distributed.run`` and ``bench.py``'s self-launch set it) or when
``ATPU_CPU_AFFINITY=1``; ``ATPU_CPU_AFFINITY=0`` turns it off. A single bare process keeps
the whole machine (its thread budget is then its allowed set, capped at 16).
"""
from __future__ import annotations

import os
import sys
from typing import Any, Dict, List, Optional, Sequence

KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"
NODE_ROOT = "/sys/devices/system/node"
DRM_ROOT = "/sys/class/drm"
MAX_THREADS = 16  # the box's CPU share per GPU; also where the stager / copy loops stop scaling

_PLAN: Optional[Dict[str, Any]] = None


def parse_cpulist(text: str) -> List[int]:
    """``"0-3,8,10-11"`` -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def _props(path: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    try:
        with open(path) as f:
            for line in f:
                kv = line.split()
                if len(kv) >= 2:
                    out[kv[0]] = kv[1]
    except OSError:
        pass
    return out


def _numeric_dirs(path: str) -> List[str]:
    try:
        return sorted((d for d in os.listdir(path) if d.isdigit()), key=int)
    except OSError:
        return []


def gpu_numa_nodes(kfd_root: Optional[str] = None, drm_root: Optional[str] = None) -> List[int]:
    """NUMA node of every GPU in KFD (= HIP enumeration) order; -1 where unknown."""
    kfd_root = kfd_root or os.getenv("ATPU_KFD_TOPOLOGY", KFD_TOPOLOGY)
    nodes = _numeric_dirs(kfd_root)
    props = {n: _props(os.path.join(kfd_root, n, "properties")) for n in nodes}
    cpu_nodes = [n for n in nodes if int(props[n].get("simd_count", "0") or 0) == 0
                 and int(props[n].get("cpu_cores_count", "0") or 0) > 0]
    numa_of_cpu_node = {n: i for i, n in enumerate(cpu_nodes)}
    out: List[int] = []
    for n in nodes:
        if int(props[n].get("simd_count", "0") or 0) == 0:
            continue
        numa = -1
        links = os.path.join(kfd_root, n, "io_links")
        for l in _numeric_dirs(links):
            to = _props(os.path.join(links, l, "properties")).get("node_to")
            if to in numa_of_cpu_node:
                numa = numa_of_cpu_node[to]
                break
        out.append(numa)
    if out and all(x >= 0 for x in out):
        return out
    # fallback: the PCI device's numa_node of every amdgpu card, in card order
    drm_root = drm_root or os.getenv("ATPU_DRM_ROOT", DRM_ROOT)
    try:
        cards = sorted((c for c in os.listdir(drm_root) if c.startswith("card") and c[4:].isdigit()),
                       key=lambda c: int(c[4:]))
    except OSError:
        cards = []
    pci: List[int] = []
    for c in cards:
        dev = os.path.join(drm_root, c, "device")
        try:
            with open(os.path.join(dev, "vendor")) as f:
                if f.read().strip().lower() != "0x1002":
                    continue
            with open(os.path.join(dev, "numa_node")) as f:
                pci.append(max(-1, int(f.read().strip())))
        except (OSError, ValueError):
            continue
    if pci and (not out or len(pci) == len(out)):
        return [p if o < 0 else o for p, o in zip(pci, out or pci)]
    return out


def node_cpus(node: int, node_root: Optional[str] = None) -> List[int]:
    node_root = node_root or os.getenv("ATPU_NODE_ROOT", NODE_ROOT)
    try:
        with open(os.path.join(node_root, f"node{node}", "cpulist")) as f:
            return parse_cpulist(f.read())
    except (OSError, ValueError):
        return []


def _visible(numa: List[int]) -> List[int]:
    """The NUMA list restricted / re-ordered by HIP_VISIBLE_DEVICES-style variables."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        raw = os.getenv(var)
        if raw is None:
            continue
        try:
            keep = [int(x) for x in raw.split(",") if x.strip()]
        except ValueError:
            continue
        return [numa[i] for i in keep if 0 <= i < len(numa)]
    return numa


def _chunk(cpus: Sequence[int], k: int, i: int) -> List[int]:
    """Chunk i of k contiguous, disjoint, near-equal chunks of ``cpus`` (never empty while
    len(cpus) >= k; with fewer cpus than chunks, chunks share cpus round robin)."""
    cpus = list(cpus)
    if not cpus:
        return []
    if len(cpus) < k:
        return [cpus[i % len(cpus)]]
    lo, hi = len(cpus) * i // k, len(cpus) * (i + 1) // k
    return cpus[lo:hi]


def plan_rank(local_rank: int, local_world: int, allowed: Sequence[int],
              numa: Optional[List[int]] = None, node_root: Optional[str] = None) -> Dict[str, Any]:
    """The cpuset and thread budget of ``local_rank`` of ``local_world`` ranks on this node.

    Rank r drives visible GPU ``r % n_gpus`` (``launch.bind_local_device``: the gloo
    rehearsal folds ranks onto fewer GPUs); the ranks whose GPUs sit on one NUMA node split
    that node's allowed cores in rank order."""
    allowed = sorted(set(allowed))
    numa = _visible(gpu_numa_nodes()) if numa is None else numa
    n_gpu = len(numa)
    if n_gpu == 0 or local_world < 1:
        cpus = _chunk(allowed, max(1, local_world), local_rank)
        return {"numa": -1, "cpus": cpus, "threads": max(1, min(MAX_THREADS, len(cpus))), "source": "even"}
    node_of = [numa[r % n_gpu] for r in range(local_world)]
    me = node_of[local_rank]
    peers = [r for r in range(local_world) if node_of[r] == me]
    node_set = [c for c in node_cpus(me, node_root) if c in set(allowed)] if me >= 0 else []
    if len(node_set) >= len(peers):
        cpus = _chunk(node_set, len(peers), peers.index(local_rank))
        src = "numa"
    else:  # unknown node, or the container does not allow its cores: even split of what it allows
        cpus = _chunk(allowed, local_world, local_rank)
        src = "even"
    return {"numa": me, "cpus": cpus, "threads": max(1, min(MAX_THREADS, len(cpus))), "source": src}


def _enabled(local_world: int) -> bool:
    mode = os.getenv("ATPU_CPU_AFFINITY", "auto").strip().lower()
    if mode in ("0", "off", "false", "no"):
        return False
    if mode in ("1", "on", "true", "yes"):
        return True
    return local_world > 1


def place_rank(apply: bool = True) -> Optional[Dict[str, Any]]:
    """Compute (and with ``apply``, set) this rank's placement; idempotent. None when off."""
    global _PLAN
    if _PLAN is not None:
        return _PLAN
    local_rank = int(os.getenv("LOCAL_RANK", "0") or 0)
    local_world = int(os.getenv("LOCAL_WORLD_SIZE", "0") or 0) or 1
    if not _enabled(local_world) or not hasattr(os, "sched_getaffinity"):
        return None
    try:
        allowed = sorted(os.sched_getaffinity(0))
        plan = plan_rank(local_rank, local_world, allowed)
    except Exception as exc:  # placement is an optimisation: never fatal
        print(f"[atpu] rank placement skipped: {exc}", file=sys.stderr, flush=True)
        return None
    plan.update(local_rank=local_rank, local_world=local_world)
    if apply and plan["cpus"]:
        try:
            os.sched_setaffinity(0, plan["cpus"])
        except OSError as exc:
            plan["error"] = str(exc)
        n = str(plan["threads"])
        # torch.distributed.run exports OMP_NUM_THREADS=1 to every rank unless the operator set
        # it (its "not tuned" default): replace that placeholder by this rank's share
        if "OMP_NUM_THREADS" not in os.environ or (os.environ["OMP_NUM_THREADS"] == "1"
                                                   and "TORCHELASTIC_RUN_ID" in os.environ):
            os.environ["OMP_NUM_THREADS"] = n
        os.environ.setdefault("ATPU_HOST_THREADS", n)
        if "torch" in sys.modules:
            try:
                sys.modules["torch"].set_num_threads(plan["threads"])
            except Exception:
                pass
    _PLAN = plan
    return plan


def current_plan() -> Optional[Dict[str, Any]]:
    return _PLAN


def host_threads(cap: int = MAX_THREADS) -> int:
    """Host thread budget of this rank for its native pools (CSV stager, risk copy threads):
    ``ATPU_HOST_THREADS`` (set by :func:`place_rank`), else the CPUs this process may run on,
    capped at ``cap``."""
    raw = os.getenv("ATPU_HOST_THREADS", "").strip()
    if raw.isdigit() and int(raw) > 0:
        return min(int(raw), cap)
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 4
    return max(1, min(cap, n))
