#!/bin/bash
# summarize defaults after the 3-stream split: decode tests, T5 1024 x2, BART 1024, T5 256.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/summdef
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 400 python -u bench/summarize.py --docs 1024 --steps 2 > $O/t5_1024_$r.log 2>&1 || exit $?
  echo "t5 1024 r$r $(grep -o '"value": [0-9.]*' $O/t5_1024_$r.log)"
done
timeout -k 10 400 python -u bench/summarize.py --docs 1024 --steps 2 --model bart-large-cnn > $O/bart_1024.log 2>&1 && echo "bart 1024 $(grep -o '"value": [0-9.]*' $O/bart_1024.log)" \
 && timeout -k 10 300 python -u bench/summarize.py --docs 256 > $O/t5_256.log 2>&1 && echo "t5 256 $(grep -o '"value": [0-9.]*' $O/t5_256.log)"
