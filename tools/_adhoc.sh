set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/kernels/test_kernels_gpu.py -x -q -k "reduce" > gpurun_out/pytest_red.log 2>&1 || { tail -40 gpurun_out/pytest_red.log; exit 1; }
tail -2 gpurun_out/pytest_red.log
timeout -k 10 300 python bench/risk_scaling.py > gpurun_out/risk.log 2>&1 || { tail -30 gpurun_out/risk.log; exit 1; }
tail -1 gpurun_out/risk.log | cut -c1-500
timeout -k 10 300 python bench/risk_scaling.py --dtype f32 > gpurun_out/risk32.log 2>&1 || { tail -30 gpurun_out/risk32.log; exit 1; }
tail -1 gpurun_out/risk32.log | cut -c1-500
