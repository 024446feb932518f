set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
MI355X_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d $GRAFT_REPO_ROOT/gpurun_out/trace -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/trace.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/trace.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/trace.log
