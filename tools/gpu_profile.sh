#!/bin/bash
# Kernel microbench + rocprofv3 kernel-trace/stats of the bench (no PMC here).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_kernels.py ${KB_ARGS:-} > gpurun_out/bench_kernels.log 2>&1
rc=$?; cat gpurun_out/bench_kernels.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log; exit $rc
