set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/kernels -x -q -m gpu > gpurun_out/pytest_k.log 2>&1 || { tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -2 gpurun_out/pytest_k.log
timeout -k 10 300 python tools/gemm_ablate.py > gpurun_out/abl0.log 2>&1 || { tail -30 gpurun_out/abl0.log; exit 1; }
tail -1 gpurun_out/abl0.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
