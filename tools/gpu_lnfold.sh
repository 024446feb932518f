#!/bin/bash
# Decode LayerNorm folding (BART): numerics tests, then BART summarize A/B (fold on / off, interleaved).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lnfold
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  ATPU_DEC_LN_FOLD=0 timeout -k 10 300 python -u bench/summarize.py --docs 256 --model bart-large-cnn > $O/off_$r.log 2>&1 || exit $?
  echo "off_$r $(grep -o '"value": [0-9.]*' $O/off_$r.log)"
  ATPU_DEC_LN_FOLD=1 timeout -k 10 300 python -u bench/summarize.py --docs 256 --model bart-large-cnn > $O/on_$r.log 2>&1 || exit $?
  echo "on_$r $(grep -o '"value": [0-9.]*' $O/on_$r.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 $R/bench/summarize.py --docs 256 --steps 1 --warmup 1 --model bart-large-cnn > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
exit $rc
