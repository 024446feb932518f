#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/kernels/test_decode_gpu.py > gpurun_out/adhoc_tests.log 2>&1 || { tail -30 gpurun_out/adhoc_tests.log; exit 1; }
tail -2 gpurun_out/adhoc_tests.log
for m in t5-base bart-large-cnn t5-base bart-large-cnn; do
echo "$m $(timeout -k 10 300 python bench/summarize.py --docs 256 --model $m 2>&1 | grep -v amdgpu.ids | cut -c1-150)" || exit 1
done
timeout -k 10 300 python tools/host_prof_summ.py bart-large-cnn 256 2>&1 | grep -v amdgpu.ids
