#!/bin/bash
# LN-folding check: epilogue + BERT GPU tests, A/B bench (fold on/off/on), serial kernel profile of the fold build.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/kernels/test_ln_fold_gpu.py tests/kernels/test_bert_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fold_tests.log 2>&1
rc=$?; tail -20 gpurun_out/fold_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_fold.log 2>&1 || exit $?
ATPU_LN_FOLD=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_nofold.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_fold2.log 2>&1 || exit $?
grep -h metric gpurun_out/bench_fold.log gpurun_out/bench_nofold.log gpurun_out/bench_fold2.log | cut -c1-160
PROF_A="ATPU_LN_FOLD=1" PROF_B="ATPU_LN_FOLD=0" bash tools/gpu_prof_ab.sh
