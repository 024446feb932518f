#!/bin/bash
# ad-hoc GPU step: concurrent-stream summarize tests + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/kernels/test_decode_gpu.py -k "concurrent or stream_split or device_select" > gpurun_out/adhoc_tests.log 2>&1 || { tail -30 gpurun_out/adhoc_tests.log; exit 1; }
tail -2 gpurun_out/adhoc_tests.log
CMD="python bench/summarize.py --docs 256" A="ATPU_SUMM_STREAMS=1" B="ATPU_SUMM_STREAMS=2" ROUNDS=2 bash tools/ab_env.sh || exit 1
CMD="python bench/summarize.py --docs 256 --model bart-large-cnn" A="ATPU_SUMM_STREAMS=1" B="ATPU_SUMM_STREAMS=2" ROUNDS=1 bash tools/ab_env.sh || exit 1
CMD="python bench/summarize.py --docs 1024" A="ATPU_SUMM_STREAMS=1" B="ATPU_SUMM_STREAMS=2" ROUNDS=1 bash tools/ab_env.sh
