#!/bin/bash
# 1024 docs/step: concurrent searches on 2 / 3 streams (ATPU_SUMM_STREAMS), interleaved, 3 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/summstreams
mkdir -p $O
for r in 1 2 3; do
  for n in 2 3; do
    ATPU_SUMM_STREAMS=$n ATPU_SUMM_PART_MIN=300 timeout -k 10 400 python -u bench/summarize.py --docs 1024 --steps 2 > $O/t5_${n}_$r.log 2>&1 || exit $?
    echo "t5 1024 streams=$n r$r $(grep -o '"value": [0-9.]*' $O/t5_${n}_$r.log)"
  done
done
