#!/bin/bash
# Headline bench at several batch sizes (rows per GPU per step), interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/abbatch
for r in 1 2; do
  for b in 1024 2048 512 4096; do
    timeout -k 10 300 python -u bench.py --batch-rows $b --steps $((20480 / b)) --warmup 3 > gpurun_out/abbatch/b${b}_r${r}.log 2>&1 || exit $?
    echo "batch=$b round=$r $(grep -o '"value": [0-9.]*' gpurun_out/abbatch/b${b}_r${r}.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abbatch/b${b}_r${r}.log)"
  done
done
