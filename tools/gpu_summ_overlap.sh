#!/bin/bash
# word-map overlap A/B (ATPU_SUMM_MAPS_OVERLAP 0/1, interleaved): T5 256 docs, BART 256 docs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/summov
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    ATPU_SUMM_MAPS_OVERLAP=$v timeout -k 10 300 python -u bench/summarize.py --docs 256 > $O/t5_${v}_$r.log 2>&1 || exit $?
    echo "t5 overlap=$v r$r $(grep -o '"value": [0-9.]*' $O/t5_${v}_$r.log)"
  done
done
for v in 0 1; do
  ATPU_SUMM_MAPS_OVERLAP=$v timeout -k 10 300 python -u bench/summarize.py --docs 256 --model bart-large-cnn > $O/bart_$v.log 2>&1 || exit $?
  echo "bart overlap=$v $(grep -o '"value": [0-9.]*' $O/bart_$v.log)"
done
