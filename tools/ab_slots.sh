#!/bin/bash
# Headline bench: serial (one compute stream) vs 2 / 3 batches in flight, interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/abslots
for r in 1 2; do
  for cfg in "serial:ATPU_CONCURRENT_SLOTS=0:2" "conc2:ATPU_CONCURRENT_SLOTS=1:2" "conc3:ATPU_CONCURRENT_SLOTS=1:3"; do
    IFS=: read name envs slots <<< "$cfg"
    env $envs timeout -k 10 300 python -u bench.py --slots $slots --steps 20 --warmup 5 > gpurun_out/abslots/${name}_r${r}.log 2>&1 || exit $?
    echo "$name round=$r $(grep -o '"value": [0-9.]*' gpurun_out/abslots/${name}_r${r}.log)"
  done
done
