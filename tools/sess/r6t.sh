# 256-doc summarize: 2 parts of 128 vs 3 parts of ~85
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=parts3_t5 ROUNDS=2 T=400 CMD="python -u bench/summarize.py --docs 256 --steps 2" A="ATPU_SUMM_PART_MIN=128" B="ATPU_SUMM_PART_MIN=80" CUT=200 bash tools/ab.sh && \
ABN=parts3_bart ROUNDS=2 T=400 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2" A="ATPU_SUMM_PART_MIN=128" B="ATPU_SUMM_PART_MIN=80" CUT=200 bash tools/ab.sh
