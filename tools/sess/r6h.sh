# decode_advance also embeds the next tokens: decode tests, 1-doc A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6h
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu > gpurun_out/r6h/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6h/tests.log
[ $rc -eq 0 ] || exit $rc
ABN=ae_t5 ROUNDS=3 T=300 CMD="python -u bench/summarize.py --docs 1 --steps 20 --warmup 3" A="ATPU_ADVANCE_EMBED=0" B="ATPU_ADVANCE_EMBED=1" CUT=250 bash tools/ab.sh && \
ABN=ae_bart ROUNDS=3 T=300 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 1 --steps 20 --warmup 3" A="ATPU_ADVANCE_EMBED=0" B="ATPU_ADVANCE_EMBED=1" CUT=250 bash tools/ab.sh
