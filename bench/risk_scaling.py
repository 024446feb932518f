#!/usr/bin/env python3
"""risk_accumulate streaming reduce (BASELINE config 5), 1..N GPUs.

Each rank holds its contiguous shard of N fp64 values resident in HBM (the
288 GB-per-GPU sizing: ``--values-per-gpu`` defaults to 256 M = 2 GiB per
rank), runs the K12 grid-stride count/sum/min/max kernel and joins the C3
RCCL all-reduces (SUM of {count,sum}, MAX of {max,-min}). A step = one full
reduction of every value. Launch with torchrun for N>1.

Baseline: SURVEY.md §6 B6 (reference ``risk_accumulate`` on CPU, 8.0 M values/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE_VALUES_PER_SEC = 8.0e6


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--values-per-gpu", type=int, default=256 * 1024 * 1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--dist-backend", default=os.environ.get("BENCH_DIST_BACKEND", "nccl"))
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group(a.dist_backend, **({"device_id": dev} if a.dist_backend == "nccl" else {}))

    from agent_tpu_amd.ops.reduce import reduce_stats_tensor
    from agent_tpu_amd.parallel.dp import comm_device

    dt = torch.float64 if a.dtype == "f64" else torch.float32
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.rand(a.values_per_gpu, generator=g, device=dev, dtype=dt)
    cdev = comm_device(dev)

    def step():
        s = reduce_stats_tensor(x)
        if world > 1:
            s = s.to(cdev)
            sums = s[:2].clone()
            ext = torch.stack([s[3], -s[2]])
            dist.all_reduce(sums)
            dist.all_reduce(ext, op=dist.ReduceOp.MAX)
            s = torch.stack([sums[0], sums[1], -ext[1], ext[0]])
        return s

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    s = s.cpu().tolist()
    assert int(s[0]) == a.values_per_gpu * world
    total = a.values_per_gpu * world * a.steps
    if rank == 0:
        bytes_per = 8 if dt == torch.float64 else 4
        print(json.dumps({
            "metric": "risk_accumulate values/sec (whole node)", "value": round(total / el, 1), "unit": "values/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el * 1000 / a.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": round(total / el / BASELINE_VALUES_PER_SEC, 1),
            "dtype": a.dtype, "data": "synthetic uniform values resident in HBM",
            "config": {"values_per_gpu": a.values_per_gpu, "parallelism": f"dp{world}",
                       "hbm_gb_per_s_per_gpu": round(a.values_per_gpu * bytes_per * a.steps / el / 1e9, 1),
                       "mean": s[1] / s[0]},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
