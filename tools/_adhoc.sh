set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/kernels/test_decode_gpu.py tests/kernels/test_bert_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench/summarize.py --docs 64 --steps 2 --warmup 1 > gpurun_out/summ.log 2>&1 || { tail -30 gpurun_out/summ.log; exit 1; }
tail -1 gpurun_out/summ.log
timeout -k 10 400 python bench/summarize.py --docs 256 --steps 2 --warmup 1 > gpurun_out/summ256.log 2>&1 || { tail -30 gpurun_out/summ256.log; exit 1; }
tail -1 gpurun_out/summ256.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_summ4 -o summ -- python3 $GRAFT_REPO_ROOT/bench/summarize.py --docs 256 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_summ4.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_summ4.log; exit 1; }
