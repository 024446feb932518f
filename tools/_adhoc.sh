#!/bin/bash
set -o pipefail
CMD="python bench/summarize.py --docs 256 --model bart-large-cnn" A="ATPU_DEC_SELF_ITEM=0" B="ATPU_DEC_SELF_ITEM=1" ROUNDS=2 CUT=150 bash tools/ab_env.sh || exit 1
CMD="python bench/summarize.py --docs 256" A="ATPU_DEC_SELF_ITEM=0" B="ATPU_DEC_SELF_ITEM=1" ROUNDS=2 CUT=150 bash tools/ab_env.sh
