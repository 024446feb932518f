#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/kernels/test_decode_gpu.py > gpurun_out/adhoc_tests.log 2>&1 || { tail -30 gpurun_out/adhoc_tests.log; exit 1; }
tail -2 gpurun_out/adhoc_tests.log
CMD="python bench/summarize.py --docs 256" ROUNDS=2 bash tools/ab_so.sh || exit 1
CMD="python bench/summarize.py --docs 256 --model bart-large-cnn" ROUNDS=2 bash tools/ab_so.sh
