#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -k "topk or device_select or concurrent" > gpurun_out/adhoc_tests.log 2>&1 || { tail -30 gpurun_out/adhoc_tests.log; exit 1; }
tail -2 gpurun_out/adhoc_tests.log
for r in 1 2; do
echo "$(timeout -k 10 300 python bench/summarize.py --docs 256 --model bart-large-cnn 2>&1 | grep -v amdgpu.ids | cut -c1-150)" || exit 1
done
