#!/bin/bash
# A/B of batch concurrency (compute streams per staging slot) on the headline bench.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/ab_concurrent.log
: > $out
run() {  # label env... -- args
  local label=$1; shift
  echo "== $label" >> $out
  env "$@" timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 3 >> $out 2>&1 || { echo "FAILED $label"; tail -5 $out; exit 1; }
  tail -1 $out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
run serial ATPU_CONCURRENT_SLOTS=0 BENCH_SLOTS=2
run conc2 ATPU_CONCURRENT_SLOTS=1 BENCH_SLOTS=2
run conc3 ATPU_CONCURRENT_SLOTS=1 BENCH_SLOTS=3
run conc2_b512 ATPU_CONCURRENT_SLOTS=1 BENCH_SLOTS=2 BENCH_BATCH_ROWS=512
done
