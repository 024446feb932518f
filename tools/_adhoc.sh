set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/kernels/test_kernels_gpu.py -x -q -k gemm > gpurun_out/pytest_gemm.log 2>&1 || { tail -40 gpurun_out/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/pytest_gemm.log
timeout -k 10 300 python tools/bench_kernels.py --only gemm_qkv,gemm_o_res,gemm_ffn1_gelu,gemm_ffn2_res --variants --rounds 5 > gpurun_out/bk.log 2>&1 || { tail -30 gpurun_out/bk.log; exit 1; }
grep -v JSON gpurun_out/bk.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
