# T5 1-doc: the cross-query GEMV prefetches the split cross attention's K/V lines: decode tests (on), A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6o
ATPU_XKV_PREFETCH=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu > gpurun_out/r6o/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6o/tests.log
[ $rc -eq 0 ] || exit $rc
ABN=xkv_t5 ROUNDS=3 T=300 CMD="python -u bench/summarize.py --docs 1 --steps 20 --warmup 3" A="ATPU_XKV_PREFETCH=0" B="ATPU_XKV_PREFETCH=1" CUT=250 bash tools/ab.sh
