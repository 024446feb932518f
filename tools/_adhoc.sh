#!/bin/bash
set -o pipefail
CMD="python bench/summarize.py --docs 256" A="ATPU_SUMM_STREAMS=1" B="ATPU_SUMM_STREAMS=2 ATPU_SUMM_PART_MIN=128" ROUNDS=2 CUT=150 bash tools/ab_env.sh || exit 1
CMD="python bench/summarize.py --docs 256 --model bart-large-cnn" A="ATPU_SUMM_STREAMS=1" B="ATPU_SUMM_STREAMS=2 ATPU_SUMM_PART_MIN=128" ROUNDS=1 CUT=150 bash tools/ab_env.sh || exit 1
CMD="python bench/summarize.py --docs 1024" A="ATPU_SUMM_STREAMS=1" B="ATPU_SUMM_STREAMS=2" ROUNDS=1 CUT=150 bash tools/ab_env.sh
