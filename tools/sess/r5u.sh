# dec kernel L2 prefetch (issued after the first K-tile barrier): decode tests, T5 summarize A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5u
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu > gpurun_out/r5u/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5u/tests.log
[ $rc -eq 0 ] || exit $rc
ABN=decpf2 ROUNDS=2 T=400 CUT=300 CMD="python -u bench/summarize.py --docs 256 --steps 2" A="ATPU_DEC_PREFETCH=0" B="ATPU_DEC_PREFETCH=1" bash tools/ab.sh
