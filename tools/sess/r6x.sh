# 1024-doc summarize: 3 vs 4 concurrent searches
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=str4_t5 ROUNDS=2 T=500 CMD="python -u bench/summarize.py --docs 1024 --steps 1" A="ATPU_SUMM_STREAMS=3" B="ATPU_SUMM_STREAMS=4" CUT=200 bash tools/ab.sh && \
ABN=str4_bart ROUNDS=1 T=500 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 1024 --steps 1" A="ATPU_SUMM_STREAMS=3" B="ATPU_SUMM_STREAMS=4" CUT=200 bash tools/ab.sh
