"""The production extension carries no timing-only code paths.

The GEMM ablations (skipped epilogues / stores, results wrong), the retired 256b / 256s
schedules, the wave-specialised kernels and the persistent decode-FFN prototype are gone
from the tree (git history and docs/PERF_NOTES.md keep the record); the retired schedules
cannot be selected.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_release_build_has_no_ablations(nat):
    for name in ("gemm_ablate", "DEV_BUILD", "qkv_attention_ws", "t5_ffn_fused", "decode_xattn_prefetch"):
        assert not hasattr(nat, name), name
    for v in (0, 2):
        with pytest.raises(ValueError, match="schedules"):
            nat.gemm_256_variant(v)
    assert nat.gemm_256_variant(-1) == 4


def test_retired_schedule_env_is_inert_in_a_fresh_process():
    code = "from agent_tpu_amd._native import native; n = native(); print(n.gemm_256_variant(-1))"
    env = dict(os.environ, ATPU_GEMM_256="b", ATPU_NO_AUTOBUILD="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["4"]


def test_no_dev_only_sources():
    kern = os.path.join(REPO, "agent_tpu_amd", "csrc")
    for root, _, files in os.walk(kern):
        for f in files:
            if f.endswith((".hip", ".cpp", ".h")):
                with open(os.path.join(root, f)) as fh:
                    assert "ATPU_DEV_BUILD" not in fh.read(), f


def test_no_binaries_tracked():
    out = subprocess.run(["git", "ls-files"], cwd=REPO, capture_output=True, text=True).stdout.split()
    bad = []
    for f in out:
        p = os.path.join(REPO, f)
        if os.path.isfile(p):
            with open(p, "rb") as fh:
                if fh.read(4) == b"\x7fELF":
                    bad.append(f)
    assert bad == []
