#!/bin/bash
# One GPU-box session: numerics tests -> smoke -> short bench. Stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
STAGE=${1:-all}
echo "[gpu_round] $(date) stage=$STAGE"
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -5 gpurun_out/smoke.log; [ $rc -ne 0 ] && { echo "smoke rc=$rc"; exit $rc; }
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; tail -5 gpurun_out/bench.log; exit $rc
