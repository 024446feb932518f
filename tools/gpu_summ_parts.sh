#!/bin/bash
# 256 docs/step as one search vs two concurrent 128-doc searches (ATPU_SUMM_PART_MIN=128), interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/summparts
mkdir -p $O
for r in 1 2; do
  for pm in 512 128; do
    ATPU_SUMM_PART_MIN=$pm timeout -k 10 300 python -u bench/summarize.py --docs 256 > $O/t5_${pm}_$r.log 2>&1 || exit $?
    echo "t5 part_min=$pm r$r $(grep -o '"value": [0-9.]*' $O/t5_${pm}_$r.log)"
  done
done
for pm in 512 128; do
  ATPU_SUMM_PART_MIN=$pm timeout -k 10 300 python -u bench/summarize.py --docs 256 --model bart-large-cnn > $O/bart_$pm.log 2>&1 || exit $?
  echo "bart part_min=$pm $(grep -o '"value": [0-9.]*' $O/bart_$pm.log)"
done
