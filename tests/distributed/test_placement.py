"""Per-rank host placement (agent_tpu_amd/parallel/placement.py): a fake
two-socket, 8-GPU KFD topology gives every local rank a disjoint cpuset on its GPU's NUMA node
and a thread budget of its share, under both launch forms (an external torch.distributed.run,
and a self-launch through launch.self_launch)."""
import json
import os
import subprocess
import sys

import pytest

from agent_tpu_amd.parallel import placement

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def fake_topology(root, cpus_per_node=(range(0, 64), range(64, 128)), gpus_per_node=4):
    """KFD nodes 0-1 = CPU sockets, 2.. = GPUs (io_link to their socket); sysfs NUMA cpulists."""
    kfd, nodes = root / "kfd", root / "node"
    for s, cpus in enumerate(cpus_per_node):
        d = kfd / str(s)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {len(cpus)}\nsimd_count 0\n")
        nd = nodes / f"node{s}"
        nd.mkdir(parents=True)
        (nd / "cpulist").write_text(f"{min(cpus)}-{max(cpus)}\n")
    g = len(cpus_per_node)
    for s in range(len(cpus_per_node)):
        for _ in range(gpus_per_node):
            d = kfd / str(g)
            (d / "io_links" / "0").mkdir(parents=True)
            (d / "properties").write_text("cpu_cores_count 0\nsimd_count 1024\nsimd_per_cu 4\n")
            (d / "io_links" / "0" / "properties").write_text(f"type 2\nnode_from {g}\nnode_to {s}\nweight 20\n")
            g += 1
    return str(kfd), str(nodes)


def test_parse_cpulist():
    assert placement.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert placement.parse_cpulist("") == []


def test_eight_ranks_two_sockets_disjoint(tmp_path, monkeypatch):
    kfd, nodes = fake_topology(tmp_path)
    monkeypatch.setenv("ATPU_KFD_TOPOLOGY", kfd)
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    numa = placement.gpu_numa_nodes()
    assert numa == [0, 0, 0, 0, 1, 1, 1, 1]
    plans = [placement.plan_rank(r, 8, range(128), numa, nodes) for r in range(8)]
    sets = [set(p["cpus"]) for p in plans]
    assert all(len(s) == 16 for s in sets) and len(set().union(*sets)) == 128  # disjoint, all cores used
    assert all(p["numa"] == (0 if r < 4 else 1) and p["source"] == "numa" for r, p in enumerate(plans))
    assert all(max(p["cpus"]) < 64 if r < 4 else min(p["cpus"]) >= 64 for r, p in enumerate(plans))
    assert [p["threads"] for p in plans] == [16] * 8
    # the container allows only part of socket 1: its ranks split what is allowed there
    plans = [placement.plan_rank(r, 8, list(range(64)) + list(range(64, 72)), numa, nodes) for r in range(8)]
    assert [len(p["cpus"]) for p in plans[4:]] == [2] * 4 and [p["threads"] for p in plans[:4]] == [16] * 4
    # the gloo rehearsal: 8 ranks folded onto ONE visible GPU share its socket 8 ways
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    numa1 = placement._visible(placement.gpu_numa_nodes())
    plans = [placement.plan_rank(r, 8, range(128), numa1, nodes) for r in range(8)]
    sets = [set(p["cpus"]) for p in plans]
    assert numa1 == [1] and all(len(s) == 8 and min(s) >= 64 for s in sets) and len(set().union(*sets)) == 64


def test_unknown_topology_splits_allowed_set(tmp_path):
    plans = [placement.plan_rank(r, 4, range(8), [], str(tmp_path)) for r in range(4)]
    assert [p["cpus"] for p in plans] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    assert all(p["source"] == "even" and p["threads"] == 2 for p in plans)


RANK_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, {repo!r})
from agent_tpu_amd.parallel.launch import ensure_rank_env
ensure_rank_env()
from agent_tpu_amd.parallel import placement
from agent_tpu_amd.runtime import risk
p = placement.current_plan() or {{}}
rec = {{"rank": int(os.environ["LOCAL_RANK"]), "aff": sorted(os.sched_getaffinity(0)), "plan": p,
        "omp": os.environ.get("OMP_NUM_THREADS"), "host": placement.host_threads(), "risk": risk._threads()}}
open(os.path.join({out!r}, "rank%d.json" % rec["rank"]), "w").write(json.dumps(rec))
"""


def _fake_env(tmp_path):
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 4:
        pytest.skip("needs 4 allowed CPUs")
    half = len(allowed) // 2
    kfd, nodes = fake_topology(tmp_path / "topo", (allowed[:half], allowed[half:2 * half]))
    env = dict(os.environ, ATPU_KFD_TOPOLOGY=kfd, ATPU_NODE_ROOT=nodes, PYTHONPATH=REPO)
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "OMP_NUM_THREADS",
              "ATPU_HOST_THREADS", "ATPU_CPU_AFFINITY", "RISK_HOST_THREADS"):
        env.pop(v, None)
    return env, allowed[:half]


def _read(out, n):
    return [json.loads((out / f"rank{r}.json").read_text()) for r in range(n)]


def _check(recs, socket0):
    affs = [set(r["aff"]) for r in recs]
    assert all(affs) and len(set().union(*affs)) == sum(len(a) for a in affs)  # disjoint
    assert all(a <= set(socket0) for a in affs)  # GPUs 0, 1 both hang off socket 0
    for r in recs:
        n = len(r["aff"])
        assert r["plan"]["source"] == "numa" and r["omp"] == str(n) and r["host"] == n and r["risk"] == n


def test_external_torchrun_ranks_are_placed(tmp_path):
    env, socket0 = _fake_env(tmp_path)
    out = tmp_path / "out"
    out.mkdir()
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT.format(repo=REPO, out=str(out)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", "0", str(script)]
    subprocess.run(cmd, env=env, check=True, timeout=180, capture_output=True)
    _check(_read(out, 2), socket0)


def test_self_launched_ranks_are_placed(tmp_path):
    env, socket0 = _fake_env(tmp_path)
    out = tmp_path / "out"
    out.mkdir()
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT.format(repo=REPO, out=str(out)))
    driver = (f"import sys; sys.path.insert(0, {REPO!r})\n"
              "from agent_tpu_amd.parallel.launch import self_launch\n"
              f"rc, _ = self_launch({str(script)!r}, [], 2)\n"
              "sys.exit(rc)\n")
    subprocess.run([sys.executable, "-c", driver], env=env, check=True, timeout=180, capture_output=True)
    _check(_read(out, 2), socket0)
