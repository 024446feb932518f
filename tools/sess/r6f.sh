# few-row LM head gated to one panel per CU: decode tests, per-call time
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6f
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu > gpurun_out/r6f/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6f/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_lm_few.py --rounds 3 > gpurun_out/r6f/lm.jsonl 2>&1; rc=$?; grep -v amdgpu gpurun_out/r6f/lm.jsonl; exit $rc
