"""Build the native `_atpu` extension in-tree with hipcc for gfx950.

Every ``kernels/*.hip``, ``runtime/*.cpp`` and ``comm/*.cpp`` translation unit plus
``bindings.cpp`` is compiled to ``build/obj`` in parallel and linked into
``agent_tpu_amd/_atpu<EXT_SUFFIX>``. Compilation is incremental (an object is
rebuilt when its source or any header is newer). No hipify, no torch headers:
kernels take raw device pointers and a hipStream_t from torch.

Usage: ``python -m agent_tpu_amd.csrc.build [--force] [--debug] [--asan-host]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List, Optional, Sequence

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
REPO = PKG.parent
BUILD = REPO / "build" / "obj"
ARCH = os.environ.get("ATPU_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def _rocm() -> str:
    return os.environ.get("ROCM_PATH", "/opt/rocm")


def _includes() -> List[str]:
    import pybind11

    return [
        f"-I{HERE / 'include'}",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
    ]


def sources() -> List[Path]:
    srcs = (sorted((HERE / "kernels").glob("*.hip")) + sorted((HERE / "runtime").glob("*.cpp"))
            + sorted((HERE / "comm").glob("*.cpp")))
    return srcs + [HERE / "bindings.cpp"]


def ext_path() -> Path:
    return PKG / ("_atpu" + sysconfig.get_config_var("EXT_SUFFIX"))


def _header_mtime() -> float:
    return max((p.stat().st_mtime for p in (HERE / "include").rglob("*.h")), default=0.0)


def _compile(src: Path, flags: List[str], force: bool) -> Path:
    obj = BUILD / (src.parent.name + "__" + src.stem + ".o")
    if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _header_mtime()):
        return obj
    cmd = [_hipcc(), *flags, "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return obj


def build(force: bool = False, debug: bool = False, asan_host: bool = False, jobs: int = 0, verbose: bool = False,
          defines: Sequence[str] = (), out: Optional[Path] = None) -> Path:
    """``defines`` + ``out``: an A/B variant of the extension (e.g. ``ATPU_GEMM_SYNC_EPI=1``)
    linked to ``out`` (load it with ``ATPU_NATIVE_PATH``), objects in their own directory."""
    global BUILD
    tag = ("_" + "_".join(d.replace("=", "") for d in defines)) if defines else ""
    BUILD = REPO / "build" / ("obj" + tag)
    BUILD.mkdir(parents=True, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result",
             "-Wno-unused-function", "-fvisibility=hidden"]
    flags += ["-O0", "-g"] if debug else ["-O3", "-DNDEBUG"]
    flags += [f"-D{d}" for d in defines]
    if asan_host:
        # host-only sanitizer: GPU ASan/xnack+ is not available on this pool
        flags += ["-Xarch_host", "-fsanitize=address", "-fno-omit-frame-pointer"]
    flags += _includes()
    srcs = sources()
    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, force), srcs))
    out = Path(out) if out is not None else ext_path()
    newest = max(o.stat().st_mtime for o in objs)
    stamp = REPO / "build" / ("linked_flavour" + tag)
    flavour = "release" + ("-debug" if debug else "") + ("-asan" if asan_host else "") + tag + str(out)
    same = stamp.exists() and stamp.read_text() == flavour
    if force or not same or not out.exists() or out.stat().st_mtime < newest:
        # librccl.so.1: at run time the copy torch already loaded (same SONAME) serves it
        link = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", str(out) + ".tmp", "-lpthread",
                f"-L{_rocm()}/lib", "-lrccl"]
        if asan_host:
            link += ["-fsanitize=address"]
        res = subprocess.run([str(x) for x in link], capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{res.stdout}\n{res.stderr}")
        os.replace(str(out) + ".tmp", out)
        stamp.write_text(flavour)
    if verbose:
        print(f"[atpu-build] {out} ({len(objs)} objects, arch {ARCH})", flush=True)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan-host", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("-D", "--define", action="append", default=[], help="A/B variant: extra -D (needs --out)")
    ap.add_argument("--out", default=None, help="A/B variant: link the extension here instead of in-tree")
    a = ap.parse_args(argv)
    if a.define and not a.out:
        ap.error("--define builds an A/B variant: give --out")
    build(force=a.force, debug=a.debug, asan_host=a.asan_host, jobs=a.jobs, verbose=True,
          defines=a.define, out=a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
