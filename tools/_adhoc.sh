#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -k "decode_attention or generate or cross" > gpurun_out/adhoc_tests.log 2>&1 || { tail -30 gpurun_out/adhoc_tests.log; exit 1; }
tail -2 gpurun_out/adhoc_tests.log
CMD="python tools/bench_xattn.py" ROUNDS=2 bash tools/ab_so.sh || exit 1
CMD="python tools/bench_xattn.py --heads 16" ROUNDS=1 bash tools/ab_so.sh || exit 1
