set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_kernels.py --only attention --rounds 7 > gpurun_out/attn_bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/attn_bench.log; exit $rc
