# fused T5 QKV + self-attention (one workgroup per head): decode tests, 1-doc T5 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6l
timeout -k 10 120 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu -k "t5_qkv_self_fused" > gpurun_out/r6l/fused.log 2>&1; rc=$?
tail -4 gpurun_out/r6l/fused.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu > gpurun_out/r6l/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6l/tests.log
[ $rc -eq 0 ] || exit $rc
ABN=qsf_t5 ROUNDS=3 T=300 CMD="python -u bench/summarize.py --docs 1 --steps 20 --warmup 3" A="ATPU_T5_QKV_SELF=0" B="ATPU_T5_QKV_SELF=1" CUT=250 bash tools/ab.sh
