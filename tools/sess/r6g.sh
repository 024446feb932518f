# beam-select record written straight into pinned host memory: decode tests, 1-doc + 256-doc A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6g
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu > gpurun_out/r6g/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6g/tests.log
[ $rc -eq 0 ] || exit $rc
ABN=zc_t5 ROUNDS=3 T=300 CMD="python -u bench/summarize.py --docs 1 --steps 20 --warmup 3" A="ATPU_REC_ZERO_COPY=0" B="ATPU_REC_ZERO_COPY=1" CUT=250 bash tools/ab.sh && \
ABN=zc_bart ROUNDS=3 T=300 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 1 --steps 20 --warmup 3" A="ATPU_REC_ZERO_COPY=0" B="ATPU_REC_ZERO_COPY=1" CUT=250 bash tools/ab.sh && \
ABN=zc_t5_256 ROUNDS=1 T=400 CMD="python -u bench/summarize.py --docs 256 --steps 2" A="ATPU_REC_ZERO_COPY=0" B="ATPU_REC_ZERO_COPY=1" CUT=250 bash tools/ab.sh
