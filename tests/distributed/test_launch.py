"""Rank launcher + device checks (VERDICT r2 'next' #1): bench.py --gpus N must
self-launch N distinct-device ranks, and no kernel may launch on another GPU's stream."""
import json
import os
import re
import subprocess
import sys
import textwrap

import pytest
import torch

from agent_tpu_amd._native import DeviceMismatch, check_launch_device
from agent_tpu_amd.parallel.launch import LaunchError, check_rank_table, self_launch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_launch_device_mismatch_raises():
    with pytest.raises(DeviceMismatch, match="cuda:1 but the current device"):
        check_launch_device(torch.device("cuda", 1), 0)
    with pytest.raises(DeviceMismatch):
        check_launch_device(torch.device("cpu"), 0)
    check_launch_device(torch.device("cuda", 3), 3)
    check_launch_device(torch.device("cuda"), 2)  # index-less = current


def test_rank_table_checks():
    t = [{"rank": 0, "device": "cuda:0", "device_id": "a"}, {"rank": 1, "device": "cuda:0", "device_id": "a"}]
    with pytest.raises(LaunchError, match="share a device"):
        check_rank_table(t, 2, "nccl")
    check_rank_table(t, 2, "gloo")  # rehearsal on one GPU is allowed
    with pytest.raises(LaunchError, match="expected 0..2"):
        check_rank_table(t, 3, "gloo")
    t[1]["device_id"] = "b"
    check_rank_table(t, 2, "nccl")


def test_self_launch_gloo(tmp_path):
    """The child torch.distributed.run starts N ranks; each verifies the group;
    rank 0's JSON line comes back to the parent."""
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import json, os, sys
        sys.path.insert(0, {REPO!r})
        import torch, torch.distributed as dist
        from agent_tpu_amd.parallel.launch import emit_result, verify_ranks
        dist.init_process_group("gloo")
        table = verify_ranks(int(sys.argv[1]), "gloo", torch.device("cpu"))
        if dist.get_rank() == 0:
            emit_result({{"world": dist.get_world_size(), "ranks": [t["rank"] for t in table],
                         "pids": len({{t["pid"] for t in table}})}})
        print("rank", dist.get_rank(), "done", flush=True)
        dist.destroy_process_group()
    """))
    rc, objs = self_launch(str(script), ["3"], 3, env={"OMP_NUM_THREADS": "1"}, timeout=120)
    assert rc == 0
    assert objs == [{"world": 3, "ranks": [0, 1, 2], "pids": 3}]


def test_self_launch_world_mismatch_fails(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {REPO!r})
        import torch, torch.distributed as dist
        from agent_tpu_amd.parallel.launch import verify_ranks
        dist.init_process_group("gloo")
        verify_ranks(4, "gloo", torch.device("cpu"))
    """))
    rc, objs = self_launch(str(script), [], 2, env={"OMP_NUM_THREADS": "1"}, timeout=120)
    assert rc != 0 and objs == []


def test_bench_refuses_more_gpus_than_visible():
    """Bare bench.py --gpus 2 under RCCL on a box without 2 GPUs exits non-zero
    before launching anything (never a silent 1-GPU number)."""
    if torch.cuda.device_count() >= 2:
        pytest.skip("box has >= 2 GPUs")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 3, r.stderr
    assert "RCCL needs one GPU per rank" in r.stderr
    assert not r.stdout.strip()


def test_bench_world_size_mismatch_exits():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 5 and "WORLD_SIZE 1" in r.stderr
    assert not any(line.startswith("{") for line in r.stdout.splitlines())


def test_health_merge_per_rank():
    from agent_tpu_amd.runtime import health

    a = {"ok": True, "devices": [{"index": 1}], "healthy": [1], "unhealthy": {}}
    b = {"ok": False, "devices": [{"index": 0}], "healthy": [], "unhealthy": {0: "GEMM probe mismatch"}}
    m = health.merge([a, b])
    assert m["healthy"] == [1] and m["unhealthy"] == {0: "GEMM probe mismatch"} and m["ok"]
    assert [d["index"] for d in m["devices"]] == [0, 1]
    json.dumps(m)


def test_probe_vram_sysfs(tmp_path):
    from worker_sizing import probe_vram

    for i, (used, tot) in enumerate([(5 << 30, 288 << 30), (7 << 30, 288 << 30)]):
        d = tmp_path / f"card{i}" / "device"
        d.mkdir(parents=True)
        (d / "vendor").write_text("0x1002\n")
        (d / "mem_info_vram_used").write_text(f"{used}\n")
        (d / "mem_info_vram_total").write_text(f"{tot}\n")
    (tmp_path / "card0-DP-1").mkdir()
    assert probe_vram(str(tmp_path)) == [(5 << 30, 288 << 30), (7 << 30, 288 << 30)]


_ENV_PROBE = """
import json, os, sys
os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None) if os.environ.get("ATPU_PROBE_CLEAR") == "1" else None
sys.path.insert(0, {repo!r})
import importlib.util
spec = importlib.util.spec_from_file_location("entry", os.path.join({repo!r}, {entry!r}))
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)  # module import only: main() is not run
from agent_tpu_amd.parallel.launch import emit_result
rank = int(os.environ.get("RANK", "0"))
val = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
if rank == 0:
    emit_result({{"rank0": val}})
print(json.dumps({{"rank": rank, "val": val}}), flush=True)
"""


@pytest.mark.parametrize("entry", ["bench.py", "app.py"])
def test_rank_env_identical_under_both_launch_forms(tmp_path, entry):
    """the rank processes see HSA_ENABLE_IPC_MODE_LEGACY=0 whether the
    ranks come from the driver's external ``torch.distributed.run`` or from bench.py's
    own self-launch, even when the launching environment does not carry it."""
    from agent_tpu_amd.parallel.launch import RANK_ENV_DEFAULTS, torchrun_cmd

    assert RANK_ENV_DEFAULTS == {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    script = tmp_path / "probe.py"
    script.write_text(_ENV_PROBE.format(repo=REPO, entry=entry))
    env = {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_IPC_MODE_LEGACY"}
    env.update(OMP_NUM_THREADS="1", ATPU_PROBE_CLEAR="1", TASKS="echo")
    # external form (as the driver runs bench.py): python -m torch.distributed.run ... script
    r = subprocess.run(torchrun_cmd(str(script), [], 2), env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    # the ranks share one stdout pipe: lines of the two processes can interleave, so the
    # records are matched anywhere in the text, not per line
    vals = [json.loads(x) for x in re.findall(r'\{"rank": \d+, "val": [^}]*\}', r.stdout)]
    assert sorted(v["rank"] for v in vals) == [0, 1] and all(v["val"] == "0" for v in vals), r.stdout
    # self-launch form: the child launcher's env gets it too (and the import sets it again)
    rc, objs = self_launch(str(script), [], 2, env={"OMP_NUM_THREADS": "1", "ATPU_PROBE_CLEAR": "1",
                                                    "TASKS": "echo"}, timeout=180)
    assert rc == 0 and objs == [{"rank0": "0"}]
    # an operator's explicit value wins (setdefault)
    env2 = dict(env, ATPU_PROBE_CLEAR="0", HSA_ENABLE_IPC_MODE_LEGACY="1")
    r = subprocess.run(torchrun_cmd(str(script), [], 2), env=env2, capture_output=True, text=True, timeout=180)
    vals = [json.loads(x) for x in re.findall(r'\{"rank": \d+, "val": [^}]*\}', r.stdout)]
    assert r.returncode == 0 and len(vals) == 2 and all(v["val"] == "1" for v in vals), r.stdout + r.stderr[-1000:]
