#!/usr/bin/env python3
"""Headline benchmark: classified rows/sec (whole node), map_classify BERT-base.

Metric/config from BASELINE.json: "classified rows/sec (whole node)
map_classify BERT-base at 1/2/4/8 MI355X". One process per GPU (torchrun);
each rank streams its own row range of a synthetic CSV through the full
map_classify device pipeline:

  C++ CSV row index -> pinned double-buffer -> hipMemcpyAsync (side stream)
  -> GPU tokenizer (K1) -> BERT-base bf16 encoder (K2..K6) -> pooler + head/top-k (K7)
  -> RCCL all-gather of every rank's per-row top-k (C2)

A "step" = one batch of ``--batch-rows`` rows per GPU (S=128 tokens each,
random-init weights broadcast from rank 0 with RCCL, C1). W warmup steps,
then exactly K timed steps bracketed by barrier + synchronize; the time is the
max over ranks. Weak scaling: per-GPU work is fixed as N grows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from agent_tpu_amd.parallel.launch import ensure_rank_env  # noqa: E402

# before anything touches the GPU, in EVERY rank however it was launched (the driver's
# external torch.distributed.run or bench.py's own self-launch): see launch.RANK_ENV_DEFAULTS
ensure_rank_env()

METRIC = "classified rows/sec (whole node) map_classify BERT-base at 1/2/4/8 MI355X"
# BASELINE.md / SURVEY.md §6 reference-compute proxies at S=128, batch 32:
# B9 BERT-base 35.2 rows/s, B10 BERT-large 8.2 rows/s
BASELINE_ROWS_PER_SEC = {"bert-base": 35.2, "bert-large": 8.2}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    # default: the batch the agent serves this model with (worker_sizing.classify_batch_rows, the
    # number the worker profile advertises), so engine, advertised and benched batch agree
    ap.add_argument("--batch-rows", type=int, default=int(os.environ.get("BENCH_BATCH_ROWS", "0")))
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--topk", type=int, default=5)
    ap.add_argument("--num-labels", type=int, default=2)
    ap.add_argument("--words-per-row", type=int, default=150)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--slots", type=int, default=int(os.environ.get("BENCH_SLOTS", "2")),
                    help="staging slots = batches in flight (each on its own compute stream)")
    ap.add_argument("--csv", default="")
    # rehearsal only: "gloo" lets >1 ranks share one GPU (RCCL refuses duplicate devices)
    ap.add_argument("--dist-backend", default=os.environ.get("BENCH_DIST_BACKEND", "nccl"))
    ap.add_argument("--comm", default=os.environ.get("ATPU_COMM", "torch"), choices=["torch", "native"],
                    help="data-plane collectives: torch.distributed (ProcessGroupNCCL) or the native RcclComm")
    a = ap.parse_args()
    os.environ["ATPU_COMM"] = a.comm
    if a.batch_rows <= 0:
        from worker_sizing import classify_batch_rows, probe_kfd

        devs = probe_kfd()  # sysfs: no HIP context before the launcher has forked the ranks
        hbm = devs[0]["total_memory_bytes"] if devs else 288 * 1024 ** 3
        a.batch_rows = classify_batch_rows(hbm, a.model, a.seq_len)
    return a


def launch_ranks(a) -> int:
    """Bare ``bench.py --gpus N`` (N > 1): start N ranks as a child torch.distributed.run.

    Nothing here touches the GPU (``device_count`` does not create a context on
    this image), and the ranks run in a child process, never an exec."""
    from agent_tpu_amd.parallel.launch import self_launch, visible_device_count

    if a.dist_backend == "nccl":
        n = visible_device_count()
        if n < a.gpus:
            print(f"[bench] --gpus {a.gpus} but only {n} visible GPU(s): RCCL needs one GPU per rank "
                  f"(use --dist-backend gloo to rehearse on fewer)", file=sys.stderr, flush=True)
            return 3
    rc, objs = self_launch(os.path.abspath(__file__), sys.argv[1:], a.gpus)
    if rc != 0 or not objs:
        print(f"[bench] ranks exited with {rc} ({len(objs)} result lines)", file=sys.stderr, flush=True)
        return rc or 4
    out = objs[-1]
    out.setdefault("config", {})["launcher"] = "self (bench.py -> child torch.distributed.run)"
    print(json.dumps(out), flush=True)
    return 0


def main() -> int:
    a = parse()
    from agent_tpu_amd.parallel.launch import LaunchError, bind_local_device, emit_result, launched, verify_ranks

    if a.gpus > 1 and not launched():
        return launch_ranks(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        print(f"[bench] rank {rank}: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr, flush=True)
        return 5
    try:
        dev = bind_local_device(a.dist_backend)
    except LaunchError as exc:
        print(f"[bench] rank {rank}: {exc}", file=sys.stderr, flush=True)
        return 5
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.dist_backend)
    try:
        rank_table = verify_ranks(a.gpus, a.dist_backend if world > 1 else "nccl", dev)
    except LaunchError as exc:
        print(f"[bench] rank {rank}: {exc}", file=sys.stderr, flush=True)
        return 5
    rccl_world = dist.get_world_size() if world > 1 else 1

    from agent_tpu_amd._native import native
    from agent_tpu_amd.models.bert import config_for, init_random
    from agent_tpu_amd.parallel.dp import all_gather_rows, broadcast_pack, comm_device
    from agent_tpu_amd.runtime.classify import ClassifyEngine
    from agent_tpu_amd.utils.synthetic import write_csv

    nat = native()
    cfg = config_for(a.model, num_labels=a.num_labels)
    B = a.batch_rows
    rows_needed = (a.warmup + a.steps) * B
    csv_path = a.csv or f"/tmp/atpu_bench_r{rank}_{rows_needed}_{a.words_per_row}.csv"
    if not os.path.exists(csv_path):
        write_csv(csv_path, rows_needed, a.words_per_row, seed=1234 + rank)
    table = nat.CsvTable(csv_path)
    col = table.column_index("text")

    # weights: rank 0 builds the seeded random init on its GPU (params.rand_fill: a kernel
    # writing the ParamPack in place, no host pass or H2D copy), then one RCCL broadcast gives
    # every rank a copy (C1, the path a checkpoint load takes). The HIP context exists before
    # either clock starts, so the two timings are the init and the collective only.
    torch.empty(1, device=dev)
    torch.cuda.synchronize(dev)
    # the first launch of an in-tree kernel loads the extension's gfx950 code object (5+ MB):
    # timed on its own (one 1-element rand_fill), so weight_init_ms is the device init only
    from agent_tpu_amd._native import launch_stream, ptr

    probe = torch.empty(1, dtype=torch.float32, device=dev)
    t_c = time.perf_counter()
    nat.rand_fill(ptr(probe), 1, True, 0, 0, 1.0, 1, 1.0, launch_stream(probe))
    torch.cuda.synchronize(dev)
    code_load_ms = (time.perf_counter() - t_c) * 1000.0
    init_ms, bcast_ms = None, None
    if rank == 0:
        t_b = time.perf_counter()
        pack = init_random(cfg, seed=0, device=dev)
        torch.cuda.synchronize(dev)
        init_ms = (time.perf_counter() - t_b) * 1000.0
    else:
        from agent_tpu_amd.models.bert import param_specs
        from agent_tpu_amd.models.params import ParamPack

        pack = ParamPack(param_specs(cfg), device=dev)
    if world > 1:
        dist.barrier()
        t_b = time.perf_counter()
        pack = broadcast_pack(pack, cfg, dev)
        torch.cuda.synchronize(dev)
        bcast_ms = (time.perf_counter() - t_b) * 1000.0

    eng = ClassifyEngine(cfg, pack, dev, batch_rows=B, seq_len=a.seq_len, topk=a.topk, use_graph=not a.no_graph,
                          slots=a.slots)

    def run(start_batch: int, nbatches: int):
        idx, score, _ = eng.classify_table(table, start_batch * B, nbatches * B, col)
        if world > 1:
            idx, score = all_gather_rows(idx, score)
        return idx, score

    run(0, a.warmup)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    idx, score = run(a.warmup, a.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_rows = world * B * a.steps
    assert idx.shape[0] == total_rows, (idx.shape, total_rows)
    value = total_rows / elapsed
    if rank == 0:
        cls_only = eng.model.cls_only_last
        flops = cfg.flops_per_row_executed(a.seq_len, cls_only) * total_rows / elapsed
        out = {
            "metric": METRIC if a.model == "bert-base" else METRIC.replace("BERT-base", a.model),
            "value": round(value, 2),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1000.0 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / BASELINE_ROWS_PER_SEC[a.model], 2)
                            if a.model in BASELINE_ROWS_PER_SEC else None),
            "dtype": "bf16",
            "data": "synthetic CSV rows (random words), random-init weights",
            "config": {
                "model": a.model,
                "global_batch": B * world,
                "seq_len": a.seq_len,
                "parallelism": f"dp{world}",
                "dist_backend": a.dist_backend if world > 1 else None,
                "comm": a.comm if world > 1 else None,
                "rccl_world_size": rccl_world if a.dist_backend == "nccl" or world == 1 else None,
                "pg_world_size": rccl_world,
                "rank_devices": [t["device"] for t in rank_table],
                "rank_hosts": [t.get("host") for t in rank_table],
                "distinct_devices": len({t["device_id"] for t in rank_table}) == len(rank_table),
                "rows_per_gpu_per_step": B,
                "num_labels": cfg.num_labels,
                "topk": min(a.topk, cfg.num_labels),
                "hipgraph": not a.no_graph,
                "concurrent_batches": a.slots if eng.concurrent else 1, "cu_split": bool(eng.cu_split),
                # the first in-tree kernel launch (code-object load), rank 0's seeded init on the
                # device (kernels only), and the C1 RCCL broadcast (N > 1 only)
                "code_object_load_ms": round(code_load_ms, 2),
                "weight_init_ms": round(init_ms, 2) if init_ms is not None else None,
                "weight_broadcast_ms": round(bcast_ms, 2) if bcast_ms is not None else None,
                "weight_bytes": int(pack.nbytes),
                "last_layer_cls_only": cls_only,
                "achieved_tflops_per_gpu": round(flops / world / 1e12, 1),
                "model_equivalent_tflops_per_gpu": round(cfg.flops_per_row(a.seq_len) * total_rows / elapsed
                                                         / world / 1e12, 1),
            },
        }
        emit_result(out)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
