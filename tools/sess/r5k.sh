# wave-specialised QKV+attention: exactness tests, then timing against the 256h kernel
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5k
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/kernels/test_qkv_attention_gpu.py -m gpu > gpurun_out/r5k/tests.log 2>&1; rc=$?
tail -30 gpurun_out/r5k/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_256h.py --no-check --full-lens --only fused_qkv_attn,256h_noepi,ws_qkv_attn,ws_noepi,ws_store > gpurun_out/r5k/bench.jsonl 2>&1; rc=$?
cat gpurun_out/r5k/bench.jsonl; exit $rc
