# BART decoder input in one launch: kernel test, decode tests, 1-doc + 256-doc A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6a
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "embed" tests/kernels/test_decode_gpu.py -m gpu > gpurun_out/r6a/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6a/tests.log
[ $rc -eq 0 ] || exit $rc
ABN=emb_1doc ROUNDS=3 T=300 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 1 --steps 20 --warmup 3" A="ATPU_AB_EMB3=1" B="ATPU_AB_EMB3=0" bash tools/ab.sh && \
ABN=emb_256 ROUNDS=1 T=400 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2" A="ATPU_AB_EMB3=1" B="ATPU_AB_EMB3=0" bash tools/ab.sh
