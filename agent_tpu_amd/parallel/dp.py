"""Data-parallel map over the GPUs of one node.

One process per GPU; ``torch.distributed`` with backend ``"nccl"`` is RCCL on
ROCm (xGMI point-to-point links), ``"gloo"`` runs the same code on CPU for
tests. Collectives issued by a DP classify task:

* C1 :func:`broadcast_pack` — every parameter lives in ONE flat byte buffer
  (ParamPack), so a model load is a single broadcast (219 MB BERT-base bf16)
  pipelined by RCCL over the links instead of ~200 small ones.
* C4 :func:`broadcast_task` — the task descriptor from rank 0 (a tiny object
  broadcast; the rank-0 agent owns the HTTP loop).
* C2 :func:`all_gather_rows` — per-rank top-k rows, padded to the largest
  shard, gathered with one ``all_gather_into_tensor`` per tensor; counts are
  gathered first (4 B/rank) so ragged shards reassemble exactly.

With ``ATPU_COMM=native`` (RCCL backend) the tensor collectives run on the
native communicator of :mod:`agent_tpu_amd.parallel.rccl` (csrc/comm/rccl_comm.cpp)
instead of ProcessGroupNCCL; objects and the task descriptor stay on torch.distributed.
* C3 (risk) is the all-reduce in :func:`agent_tpu_amd.parallel.dp_ops.risk_task`.

Shard planning is contiguous and balanced (:func:`split_range`), so results
concatenate in rank order into the original row order.

Elastic recovery: :func:`shrink` drops ranks whose device
faulted. The survivors build a new process group over the healthy ranks (a
new RCCL communicator, ``use_local_synchronization`` so the lost ranks take no
part), and every collective here runs on that group. Global rank 0 (the agent)
is never dropped.
"""
from __future__ import annotations

from typing import Any, Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import watchdog


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


_GROUP = None  # active DP group after a shrink (None = the default group)
_NATIVE = None  # ATPU_COMM=native: RCCL communicator over the active group (rebuilt on shrink)
_MEMBERS: Optional[List[int]] = None  # its global ranks, ascending
_LOST: List[int] = []


def group():
    return _GROUP


def members() -> List[int]:
    """Global ranks of the active DP group."""
    if not is_dist():
        return [0]
    return list(_MEMBERS) if _MEMBERS is not None else list(range(dist.get_world_size()))


def world() -> Tuple[int, int]:
    """(rank within the active DP group, its size); rank -1 once this rank was dropped."""
    if not is_dist():
        return (0, 1)
    if _MEMBERS is None:
        return (dist.get_rank(), dist.get_world_size())
    me = dist.get_rank()
    return (_MEMBERS.index(me) if me in _MEMBERS else -1, len(_MEMBERS))


def lost_ranks() -> List[int]:
    return list(_LOST)


def shrink(lost: Iterable[int]) -> bool:
    """Drop global ranks ``lost`` from the DP group; every member calls this with
    the same set (the exchanged per-rank errors). Returns False when nothing
    changes or rank 0 would be dropped (the agent process cannot leave)."""
    global _GROUP, _MEMBERS
    cur = members()
    gone = set(lost) & set(cur)
    if not gone or 0 in gone:
        return False
    keep = [r for r in cur if r not in gone]
    _LOST.extend(sorted(gone))
    _MEMBERS = keep
    global _NATIVE
    if _NATIVE is not None:
        _NATIVE.comm.abort()  # its peers include the lost ranks; rebuilt lazily over the survivors
        _NATIVE = None
    if dist.get_rank() in keep:
        _GROUP = dist.new_group(ranks=keep, use_local_synchronization=True)
    return True


def native_comm(dev: torch.device):
    """The native RCCL communicator of the active DP group (``ATPU_COMM=native``, RCCL
    backend, device tensors), created collectively on first use; None otherwise."""
    global _NATIVE
    from . import rccl

    if not (rccl.enabled() and is_dist() and dist.get_backend() == "nccl" and dev.type == "cuda"):
        return None
    if _NATIVE is not None and not _NATIVE.healthy():
        # aborted by a failed wait (or an async error) on THIS rank only: a local rebuild would
        # be a collective its still-healthy peers never join (deadlock or mismatched
        # collectives), so the group is lost and the launcher restarts it
        _NATIVE = None
        raise watchdog.RankLost(f"rank {dist.get_rank()}: native RCCL communicator aborted")
    if _NATIVE is None:
        with watchdog.collective("rccl communicator init"):
            _NATIVE = rccl.NativeComm.from_group(dev, group=_GROUP, ranks=members())
    return _NATIVE


def split_range(start: int, n: int, world_size: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split of ``[start, start+n)``; returns (start_r, n_r)."""
    base, rem = divmod(max(0, n), world_size)
    n_r = base + (1 if rank < rem else 0)
    s_r = start + rank * base + min(rank, rem)
    return s_r, n_r


def comm_device(default: Optional[torch.device] = None) -> torch.device:
    """Device collectives must use: the local GPU for nccl(RCCL), CPU for gloo."""
    if is_dist() and dist.get_backend() == "nccl":
        return default if default is not None and default.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_pack(pack, cfg, device: torch.device, src: int = 0, builder=None):
    """C1: broadcast rank ``src``'s ParamPack buffer to every rank, on ``device``."""
    from ..models.params import ParamPack
    from ..models.bert import param_specs

    specs = builder(cfg) if builder is not None else param_specs(cfg)
    rank, _ = world()
    if rank == src:
        assert pack is not None
        out = pack if pack.buffer.device == device else pack.to(device)
    else:  # destination: preallocated by the caller (dp_ops.load_collectively) or here
        out = pack if pack is not None and pack.buffer.device == device else ParamPack(specs, device=device)
    if is_dist():
        cdev = comm_device(device)
        buf = out.buffer if out.buffer.device == cdev else out.buffer.to(cdev)
        nc = native_comm(cdev)
        with watchdog.collective("weight broadcast"):
            if nc is not None:  # C1 on the native communicator (group rank of the source)
                nc.broadcast(buf, root=members().index(src))
                nc.wait("weight broadcast")  # complete inside the bracket: hang detection
            else:
                dist.broadcast(buf, src=src, group=_GROUP)
        if buf is not out.buffer:
            out.buffer.copy_(buf)
    return out


def broadcast_task(obj: Any, src: int = 0) -> Any:
    """C4: broadcast a small picklable task descriptor from ``src``."""
    if not is_dist():
        return obj
    box = [obj]
    with watchdog.collective("task broadcast"):
        dist.broadcast_object_list(box, src=src, group=_GROUP)
    return box[0]


def all_gather_rows(*tensors: Optional[torch.Tensor], counts: Optional[List[int]] = None
                    ) -> Tuple[torch.Tensor, ...]:
    """C2: concatenate every rank's ``[rows_r, ...]`` tensors in rank order.

    Ragged shards are padded to ``max(rows_r)`` for the collective and trimmed
    afterwards using the row counts: ``counts`` when the caller already exchanged them
    (``dp_ops._check_errors(err, rows)`` carries them in its object exchange), else one
    count all-gather (4 B per rank) first.
    """
    if not is_dist():
        return tensors
    _, ws = world()
    dev = tensors[0].device
    cdev = comm_device(dev)
    nc = native_comm(cdev)
    if counts is None:
        cnt = torch.tensor([tensors[0].shape[0]], dtype=torch.int64, device=cdev)
        cts = torch.empty(ws, dtype=torch.int64, device=cdev)
        with watchdog.collective("row-count gather"):
            if nc is not None:
                nc.all_gather_into(cts, cnt)
                nc.wait("row-count gather")
            else:
                dist.all_gather_into_tensor(cts, cnt, group=_GROUP)
        counts = cts.tolist()
    counts_l: List[int] = [int(c) for c in counts]
    assert len(counts_l) == ws and counts_l[world()[0]] == tensors[0].shape[0], (counts_l, tensors[0].shape)
    mx = max(counts_l) if counts_l else 0
    outs = []
    for t in tensors:
        t = t.to(cdev)
        if t.shape[0] < mx:
            pad = torch.zeros((mx - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=cdev)
            t = torch.cat([t, pad], 0)
        t = t.contiguous()
        g = torch.empty((ws * mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=cdev)
        with watchdog.collective("row all-gather"):
            if nc is not None:
                nc.all_gather_into(g, t)
                nc.wait("row all-gather")
            else:
                dist.all_gather_into_tensor(g, t, group=_GROUP)
        if all(c == mx for c in counts_l):
            outs.append(g.to(dev))
        else:
            parts = [g[r * mx:r * mx + counts_l[r]] for r in range(ws)]
            outs.append(torch.cat(parts, 0).to(dev))
    return tuple(outs)
