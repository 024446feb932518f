"""The production extension carries no timing-only code paths.

GEMM ablations (``ATPU_GEMM_ABLATE``: skipped epilogues / stores, results wrong) and
the retired 256b / 256s schedules are compiled only with ``--dev``
(``-DATPU_DEV_BUILD``). In the release build the env var and the setter are inert and
the retired schedules cannot be selected.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_release_build_has_no_ablations(nat):
    assert nat.DEV_BUILD is False
    assert nat.gemm_ablate(4) == 0 and nat.gemm_ablate(-1) == 0
    for v in (0, 2):
        with pytest.raises(ValueError, match="dev build"):
            nat.gemm_256_variant(v)
    assert nat.gemm_256_variant(-1) == 4


def test_ablate_env_is_inert_in_a_fresh_process():
    code = ("from agent_tpu_amd._native import native; n = native(); "
            "print(n.DEV_BUILD, n.gemm_ablate(-1), n.gemm_256_variant(-1))")
    env = dict(os.environ, ATPU_GEMM_ABLATE="4", ATPU_GEMM_256="b", ATPU_NO_AUTOBUILD="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["False", "0", "4"]


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
