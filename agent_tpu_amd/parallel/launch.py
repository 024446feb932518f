"""Single-node rank launcher and rank/device verification.

``bench.py --gpus N`` (and any other entry point) can be started either by an
external ``torch.distributed.run`` (the driver's form: WORLD_SIZE is set) or
bare. Bare with N > 1, :func:`self_launch` starts ``torch.distributed.run`` as a
CHILD process (never ``exec``: the parent has not touched the GPU and must not
replace itself after anything has) and relays the ranks' output; the parent
exits with the child's code.

Inside the ranks, :func:`verify_ranks` checks the process group is what the
caller asked for: ``WORLD_SIZE == expected``, every rank bound to a device that
exists (no ``local % device_count()`` folding), and under RCCL every rank on a
DISTINCT device (RCCL over xGMI needs one GPU per rank; the gloo rehearsal may
share one). It returns the per-rank device table the bench reports.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from typing import Any, Dict, List, Optional, Sequence, Tuple


class LaunchError(RuntimeError):
    pass


# Environment every GPU rank process needs, whichever launcher started it.
#
# HSA_ENABLE_IPC_MODE_LEGACY=0: the amdgpu host driver of the MI355X pool supports only
# dmabuf-based IPC. With the legacy IPC mode the ROCr runtime's hipIpcGetMemHandle fails
# ("invalid argument"), and RCCL uses IPC handles to map its peer buffers between the
# ranks' processes (intra-node P2P transport over xGMI): communicator setup then fails.
# The variable is read when the HSA runtime initialises, i.e. at the first HIP call, so
# each entry point applies it at import, before anything touches the GPU. setdefault: an
# operator's explicit value wins.
RANK_ENV_DEFAULTS = {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}


def ensure_rank_env(env: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """Apply :data:`RANK_ENV_DEFAULTS` to ``env`` (default: this process's environment).

    Called at import by ``bench.py`` and ``app.py`` (so a rank started by an external
    ``torch.distributed.run`` gets it exactly like one started by :func:`self_launch`)
    and by :func:`self_launch` for the child launcher's environment."""
    target = os.environ if env is None else env
    for k, v in RANK_ENV_DEFAULTS.items():
        target.setdefault(k, v)
    if env is None:
        # this process is a rank: CPU affinity + host thread budget by its GPU's NUMA node
        from .placement import place_rank

        place_rank()
    return target


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launched() -> bool:
    """True inside a rank started by torch.distributed.run (or any WORLD_SIZE launcher)."""
    return "WORLD_SIZE" in os.environ


def visible_device_count() -> int:
    """GPUs this node exposes, WITHOUT creating a HIP context.

    ``torch.cuda.device_count()`` does not initialise the GPU on this image (it
    asks the driver through amdsmi / the KFD), so a parent may call it before it
    spawns its ranks."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:
        return 0


def torchrun_cmd(script: str, argv: Sequence[str], nproc: int, port: Optional[int] = None) -> List[str]:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(nproc)}",
            "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()), script, *argv]


RESULT_ENV = "ATPU_RESULT_FILE"


def emit_result(obj: Dict[str, Any]) -> None:
    """Print the rank-0 result line; under :func:`self_launch` also write it to the
    parent's result file (the ranks share one stdout pipe, where lines of different
    ranks can interleave)."""
    line = json.dumps(obj)
    print(line, flush=True)
    path = os.environ.get(RESULT_ENV)
    if path:
        with open(path + ".tmp", "w") as f:
            f.write(line + "\n")
        os.replace(path + ".tmp", path)


def self_launch(script: str, argv: Sequence[str], nproc: int, env: Optional[Dict[str, str]] = None,
                timeout: Optional[float] = None) -> Tuple[int, List[Dict[str, Any]]]:
    """Run ``script argv`` on ``nproc`` ranks as a child ``torch.distributed.run``.

    The ranks' output is relayed to stderr as it arrives (a long run keeps showing
    progress). The result is what rank 0 passed to :func:`emit_result` (a file
    named by ``ATPU_RESULT_FILE``); failing that, every stdout line that parses as
    a JSON object. Returns ``(returncode, json_objects)``."""
    import tempfile

    cmd = torchrun_cmd(script, argv, nproc)
    fd, res_path = tempfile.mkstemp(prefix="atpu_result_", suffix=".json")
    os.close(fd)
    os.unlink(res_path)
    child_env = dict(os.environ)
    child_env.update(env or {})
    child_env[RESULT_ENV] = res_path
    ensure_rank_env(child_env)  # each rank sizes OMP / host threads by its NUMA share (placement.py)
    objs: List[Dict[str, Any]] = []
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, env=child_env, text=True, bufsize=1)
    try:
        assert proc.stdout is not None
        for line in proc.stdout:
            s = line.strip()
            if s.startswith("{"):
                try:
                    obj = json.loads(s)
                except ValueError:
                    obj = None
                if isinstance(obj, dict):
                    objs.append(obj)
                    continue
            sys.stderr.write(line)
            sys.stderr.flush()
        rc = proc.wait(timeout=timeout)
    except BaseException:
        proc.kill()
        proc.wait()
        raise
    finally:
        try:
            with open(res_path) as f:
                filed = [json.loads(x) for x in f.read().splitlines() if x.strip()]
            os.unlink(res_path)
        except (OSError, ValueError):
            filed = []
    return rc, (filed or objs)


def bind_local_device(backend: str):
    """The device of this rank: ``cuda:LOCAL_RANK``, which must exist under RCCL.

    The gloo rehearsal (several ranks on a one-GPU box) maps ``LOCAL_RANK`` onto
    the visible devices round-robin and says so in :func:`verify_ranks`."""
    import torch

    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = torch.cuda.device_count()
    if n == 0:
        return torch.device("cpu")
    if local >= n:
        if backend == "nccl":
            raise LaunchError(f"LOCAL_RANK {local} but only {n} visible GPU(s): RCCL needs one GPU per rank")
        local = local % n
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    return dev


def _device_id(dev) -> str:
    import torch

    if dev.type != "cuda":
        return "cpu"
    try:
        uuid = getattr(torch.cuda.get_device_properties(dev), "uuid", None)
        if uuid is not None:
            return str(uuid)
    except Exception:
        pass
    return f"cuda:{dev.index}"


def check_rank_table(table: List[Dict[str, Any]], expected: int, backend: str) -> None:
    """Raise :class:`LaunchError` unless ``table`` (one entry per rank) is a valid
    ``expected``-rank group: ranks 0..N-1 exactly once, and under RCCL distinct devices."""
    ranks = sorted(int(t["rank"]) for t in table)
    if ranks != list(range(expected)):
        raise LaunchError(f"process group has ranks {ranks}, expected 0..{expected - 1}")
    if backend == "nccl":
        ids = [t["device_id"] for t in table]
        if len(set(ids)) != len(ids):
            raise LaunchError(f"ranks share a device under RCCL: {[(t['rank'], t['device']) for t in table]}")


def verify_ranks(expected: int, backend: str, dev) -> List[Dict[str, Any]]:
    """Collective: gather every rank's device and validate the group (all ranks raise together)."""
    import torch.distributed as dist

    ws = dist.get_world_size() if dist.is_initialized() else 1
    if ws != expected:
        raise LaunchError(f"WORLD_SIZE {ws} != --gpus {expected}")
    from .placement import current_plan, host_threads

    me = {"rank": dist.get_rank() if dist.is_initialized() else 0, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "device": str(dev), "device_id": _device_id(dev), "pid": os.getpid()}
    plan = current_plan()
    try:
        aff = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = []
    # host placement (placement.py): NUMA node, the cpuset this rank runs on, its thread budget
    me["host"] = {"numa": plan["numa"] if plan else None, "source": plan["source"] if plan else "unplaced",
                  "cpus": (f"{aff[0]}-{aff[-1]}" if aff and aff[-1] - aff[0] + 1 == len(aff) else str(len(aff)))
                  if aff else None, "ncpus": len(aff), "threads": host_threads()}
    table: List[Dict[str, Any]] = [me]
    if dist.is_initialized() and ws > 1:
        table = [None] * ws  # type: ignore[list-item]
        dist.all_gather_object(table, me)
    table.sort(key=lambda t: t["rank"])
    check_rank_table(table, expected, backend)
    return table
