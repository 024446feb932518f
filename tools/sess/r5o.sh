# ws FFN1 with the scalar GELU on the loader waves
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5o
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_gemm_ws_gpu.py -m gpu > gpurun_out/r5o/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5o/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_ffn1_ws.py --variants 104 > gpurun_out/r5o/bench.jsonl 2>&1; rc=$?
cat gpurun_out/r5o/bench.jsonl; exit $rc
