#!/bin/bash
# Headline bench sweep: batch rows x batch concurrency.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/ab_batch.log
: > $out
run() {
  local label=$1; shift
  echo "== $label" >> $out
  env "$@" timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 3 >> $out 2>&1 || { echo "FAILED $label"; tail -5 $out; exit 1; }
  tail -1 $out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
run b1024_serial ATPU_CONCURRENT_SLOTS=0 BENCH_BATCH_ROWS=1024
run b1024_conc ATPU_CONCURRENT_SLOTS=1 BENCH_BATCH_ROWS=1024
run b2048_serial ATPU_CONCURRENT_SLOTS=0 BENCH_BATCH_ROWS=2048
run b2048_conc ATPU_CONCURRENT_SLOTS=1 BENCH_BATCH_ROWS=2048
done
