set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/kernels/test_rccl_gpu.py -x -q > gpurun_out/pytest_rccl.log 2>&1 || { tail -40 gpurun_out/pytest_rccl.log; exit 1; }
tail -2 gpurun_out/pytest_rccl.log
timeout -k 10 300 python bench.py --model bert-large --steps 10 --warmup 2 > gpurun_out/bench_large.log 2>&1 || { tail -30 gpurun_out/bench_large.log; exit 1; }
tail -1 gpurun_out/bench_large.log | cut -c1-700
