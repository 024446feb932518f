#!/usr/bin/env python3
"""map_classify scaling curve (BASELINE config 3): bench.py at 1, 2, 4, ... GPUs of one node.

Each point is its own job: N=1 runs ``bench.py`` directly, N>1 under
``torch.distributed.run`` (one rank per GPU, RCCL, rendezvous on 127.0.0.1),
exactly the way the round driver launches it. Weak scaling: every rank
classifies ``--batch-rows`` rows per step, so ideal whole-node rows/s is
N x the 1-GPU value; the efficiency column is value(N) / (N * value(1)).

    python bench/classify_scaling.py --gpus 1,2,4,8 --steps 20 --warmup 3 [--model bert-large]

GPU counts above ``torch.cuda.device_count()`` are skipped. Rows are printed
as a table and the raw JSON lines are written to ``--out`` (optional).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_point(n: int, args, port: int) -> dict:
    bench = [os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", str(args.steps), "--warmup",
             str(args.warmup), "--model", args.model]
    if n == 1:
        cmd = [sys.executable] + bench
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(port)] + bench
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=args.timeout)
    if out.returncode != 0:
        raise RuntimeError(f"N={n} failed rc={out.returncode}:\n{out.stderr[-2000:]}")
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--timeout", type=int, default=900)
    ap.add_argument("--port", type=int, default=29531)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    avail = torch.cuda.device_count()
    points = []
    for i, n in enumerate(int(x) for x in a.gpus.split(",") if x):
        if n > avail:
            print(f"skip N={n}: {avail} GPU(s) visible")
            continue
        points.append(run_point(n, a, a.port + i))
    if not points:
        return 1
    base = points[0]["value"] / points[0]["n_gpus"]
    print(f"{'N':>3} {'rows/s':>12} {'ms/step':>9} {'efficiency':>10}")
    for p in points:
        eff = p["value"] / (p["n_gpus"] * base)
        print(f"{p['n_gpus']:>3} {p['value']:>12,.0f} {p['ms_per_step']:>9.2f} {eff:>10.3f}")
    if a.out:
        with open(a.out, "w") as f:
            for p in points:
                f.write(json.dumps(p) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
