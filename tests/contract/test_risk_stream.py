"""Streamed risk_accumulate over a CSV column (BASELINE config 5).

CPU side of agent_tpu_amd/runtime/risk.py: chunked native parse into one reusable buffer.
Chunk boundaries and ragged tails must give the fp64 sums of a one-pass parse, bad values
must raise the single-pass error, and peak host memory must not grow with shard_size.
The GPU path (RiskStream, device parse) is tests/kernels/test_runtime_gpu.py.
"""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _write(path, vals, header="id,risk,note"):
    with open(path, "w") as f:
        f.write(header + "\n")
        for i, v in enumerate(vals):
            f.write(f"{i},{v},n{i}\n")
    return str(path)


@pytest.fixture(scope="module")
def nat():
    from agent_tpu_amd._native import native

    return native()


def _ref(vals):
    x = np.array([float(v) for v in vals], dtype=np.float64)
    return [float(x.size), float(x.sum()), float(x.min()), float(x.max())]


@pytest.mark.parametrize("rows", [1, 7, 64, 1000, 5000])
def test_chunk_boundaries_and_ragged_tails(tmp_path, nat, rows):
    from agent_tpu_amd.runtime.risk import column_stats

    rng = np.random.default_rng(rows)
    vals = [f"{v:.6f}" for v in rng.uniform(-1000, 1000, 4321)]
    t = nat.CsvTable(_write(tmp_path / "r.csv", vals))
    col = t.column_index("risk")
    for start, n in ((0, 4321), (5, 4000), (4320, 5), (17, 1), (100, 0)):
        st, info = column_stats(t, start, n, col, None, rows=rows)
        want = _ref(vals[start:start + n]) if n and start < 4321 else [0.0, 0.0, float("inf"), float("-inf")]
        got = st.tolist()
        assert got[0] == want[0] and got[2] == want[2] and got[3] == want[3], (start, n)
        assert abs(got[1] - want[1]) <= 1e-9 * max(1.0, abs(want[1])), (got, want)
        assert info["chunks"] == (max(0, min(n, 4321 - start)) + rows - 1) // rows


def test_bad_value_raises_single_pass_error(tmp_path, nat):
    from agent_tpu_amd.runtime.risk import column_stats

    vals = ["1.5"] * 50 + ["abc"] + ["2"] * 10 + ["zzz"]
    t = nat.CsvTable(_write(tmp_path / "bad.csv", vals))
    with pytest.raises(ValueError, match="could not convert string to float: 'abc'"):
        column_stats(t, 0, len(vals), t.column_index("risk"), None, rows=8)
    with pytest.raises(ValueError) as one_pass:
        t.float_column(0, len(vals), t.column_index("risk"))
    assert "'abc'" in str(one_pass.value)


def test_op_csv_form_matches_values_form(tmp_path, monkeypatch):
    from ops.risk_accumulate import risk_accumulate

    monkeypatch.setenv("RISK_DEVICE", "cpu")
    monkeypatch.setenv("RISK_CHUNK_ROWS", "33")
    vals = [f"{(i * 37 % 1001) / 7:.5f}" for i in range(1000)]
    path = _write(tmp_path / "op.csv", vals)
    out = risk_accumulate({"source_uri": path, "field": "risk", "start_row": 10, "shard_size": 500})
    ref = risk_accumulate({"values": [float(v) for v in vals[10:510]]})
    assert out["count"] == 500 and out["min"] == ref["min"] and out["max"] == ref["max"]
    assert abs(out["sum"] - ref["sum"]) < 1e-9 * abs(ref["sum"])
    assert out["stream"]["chunks"] == 16  # ceil(500 / 33)


_RSS = """
import json, os, sys, resource
sys.path.insert(0, {repo!r})
os.environ["RISK_DEVICE"] = "cpu"
os.environ["RISK_CHUNK_ROWS"] = "65536"
from agent_tpu_amd._native import native
from agent_tpu_amd.runtime.risk import column_stats
t = native().CsvTable({path!r})
col = t.column_index("risk")
def hwm():
    for line in open("/proc/self/status"):
        if line.startswith("VmHWM:"):
            return int(line.split()[1]) * 1024
column_stats(t, 0, 1000, col, None)  # warm: code paths, allocator
base = hwm()
st, _ = column_stats(t, 0, int(sys.argv[1]), col, None)
print(json.dumps({{"delta": hwm() - base, "count": st[0].item()}}))
"""


def test_peak_host_memory_independent_of_shard_size(tmp_path):
    """Peak RSS (VmHWM, which counts the mapped file pages too) grows by about the same
    for a 0.4 M-row and a 3.2 M-row shard: one chunk buffer, consumed file pages dropped."""
    path = tmp_path / "big.csv"
    with open(path, "w") as f:
        f.write("id,risk\n")
        f.writelines(f"{i},{(i % 9973) / 13:.6f}\n" for i in range(3_200_000))
    script = tmp_path / "rss.py"
    script.write_text(_RSS.format(repo=REPO, path=str(path)))

    def run(n):
        r = subprocess.run([sys.executable, str(script), str(n)], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, OMP_NUM_THREADS="2"))
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout.strip().splitlines()[-1])

    small, big = run(400_000), run(3_200_000)
    assert small["count"] == 400_000 and big["count"] == 3_200_000
    # a one-pass parse would add 8 B x 2.8 M = 22 MB of values plus ~50 MB of mapped file
    assert big["delta"] - small["delta"] < 8 << 20, (small, big)


def test_small_shard_stays_on_host(tmp_path, monkeypatch):
    """a shard below RISK_GPU_MIN_VALUES rows is reduced on the host even when a
    device is passed (no pinned stream is built for it)."""
    import torch

    from agent_tpu_amd._native import native
    from agent_tpu_amd.runtime import risk

    path = tmp_path / "s.csv"
    path.write_text("id,risk\n" + "".join(f"{i},{i * 0.5}\n" for i in range(100)))
    t = native().CsvTable(str(path))
    monkeypatch.delenv("RISK_DEVICE", raising=False)
    monkeypatch.setenv("RISK_GPU_MIN_VALUES", "1000")
    n0 = len(risk._STREAMS)
    st, info = risk.column_stats(t, 0, 100, t.column_index("risk"), torch.device("cuda", 0))
    assert info["device"] == "cpu" and len(risk._STREAMS) == n0
    assert st.tolist() == [100.0, sum(i * 0.5 for i in range(100)), 0.0, 49.5]


def test_small_csv_shard_never_touches_hip(tmp_path, monkeypatch):
    """a CSV shard below RISK_GPU_MIN_VALUES rows is reduced without ever asking for a
    device (risk_device() initialises HIP); the row count is known from the row index first."""
    from agent_tpu_amd.parallel import dp_ops

    path = tmp_path / "s.csv"
    path.write_text("id,risk\n" + "".join(f"{i},{i * 0.25}\n" for i in range(200)))
    monkeypatch.delenv("RISK_DEVICE", raising=False)
    monkeypatch.setenv("RISK_GPU_MIN_VALUES", "1000")

    def boom():
        raise AssertionError("risk_device() called for a small shard")

    monkeypatch.setattr(dp_ops, "risk_device", boom)
    import ops.risk_accumulate as ra

    out = ra.risk_accumulate({"source_uri": str(path), "field": "risk"})
    assert out["count"] == 200 and out["sum"] == sum(i * 0.25 for i in range(200))
    assert out.get("device") != "gpu"
