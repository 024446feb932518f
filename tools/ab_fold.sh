#!/bin/bash
# Interleaved headline-bench A/B: LN folding on / off, N rounds (default 2).
set -o pipefail
mkdir -p gpurun_out/abfold
for r in $(seq 1 ${ROUNDS:-2}); do
  for f in 1 0; do
    ATPU_LN_FOLD=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/abfold/f${f}_r${r}.log 2>&1 || exit $?
    echo "fold=$f round=$r $(grep -o '"value": [0-9.]*' gpurun_out/abfold/f${f}_r${r}.log)"
  done
done
