# ws kernel variants: read scheduling fix, MMA priority, DMA-wait diagnostic
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5l
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_qkv_attention_gpu.py -m gpu -k "ws" > gpurun_out/r5l/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5l/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_256h.py --no-check --full-lens --only fused_qkv_attn,ws_qkv_attn,ws_noepi --ws-variants 8,72,104 > gpurun_out/r5l/bench.jsonl 2>&1; rc=$?
cat gpurun_out/r5l/bench.jsonl; exit $rc
