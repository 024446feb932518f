set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for A in 0 1 2 3; do echo -n "ablate=$A "; ATPU_GEMM_ABLATE=$A timeout -k 10 300 python tools/bench_kernels.py --only gemm_ffn2_res --rounds 3 2>&1 | grep -v amdgpu.ids | grep -v JSON; done
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels.log 2>&1; grep -v amdgpu gpurun_out/bench_kernels.log | grep -v JSON
timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep metric | tee gpurun_out/bench_1gpu.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1
