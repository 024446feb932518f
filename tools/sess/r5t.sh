# summarize end to end: faster flash attention; BART encoder LN fold (tests, then on / off)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5t
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu -k "ln_fold_matches_unfolded or long_source" > gpurun_out/r5t/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5t/tests.log
[ $rc -eq 0 ] || exit $rc
OUT=r5t bash tools/gpu.sh "run:s256:python -u bench/summarize.py --docs 256 --steps 2" \
  "run:b256:python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2" && \
OUT=r5t STAGE_ENV="ATPU_ENC_LN_FOLD=0" bash tools/gpu.sh "run:b256_nofold:python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2"
