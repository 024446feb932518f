"""Host C++ under AddressSanitizer + UBSan: builds
tests/native/host_sanitize.cpp against the CSV index and host tokenizer with
``-Xarch_host -fsanitize=...`` (host side only) and runs it on the CPU."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(REPO, "agent_tpu_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_host_code_is_sanitizer_clean(tmp_path):
    exe = str(tmp_path / "host_sanitize")
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined"]
    cmd = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *san,
           f"-I{CSRC}/include", os.path.join(REPO, "tests/native/host_sanitize.cpp"),
           f"{CSRC}/runtime/csv_index.cpp", f"{CSRC}/runtime/host_runtime.cpp",
           "-fsanitize=address,undefined", "-lpthread", "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-4000:]
    (tmp_path / "idx").mkdir()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               ATPU_CSV_INDEX_DIR=str(tmp_path / "idx"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "clean" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
