# T5 / BART 256-doc summarize: one search vs 2 concurrent parts of 128 (src 1024 now)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=parts_t5 ROUNDS=2 T=400 CMD="python -u bench/summarize.py --docs 256 --steps 2" A="ATPU_SUMM_PART_MIN=300" B="ATPU_SUMM_PART_MIN=128" CUT=200 bash tools/ab.sh && \
ABN=parts_bart ROUNDS=2 T=400 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2" A="ATPU_SUMM_PART_MIN=300" B="ATPU_SUMM_PART_MIN=128" CUT=200 bash tools/ab.sh
