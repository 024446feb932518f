# ws GEMM (FFN1) and ws QKV+attention: exactness tests, then A/B against the production kernels
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5n
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_gemm_ws_gpu.py tests/kernels/test_qkv_attention_gpu.py -m gpu > gpurun_out/r5n/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5n/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_ffn1_ws.py > gpurun_out/r5n/bench.jsonl 2>&1; rc=$?
cat gpurun_out/r5n/bench.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_256h.py --no-check --full-lens --only fused_qkv_attn,ws_qkv_attn --ws-variants 8,72,104 > gpurun_out/r5n/qkv.jsonl 2>&1; rc=$?
cat gpurun_out/r5n/qkv.jsonl; exit $rc
