# headline: re-check the concurrency knobs after this round's kernel changes (2 vs 3 slots; CU split)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=slots3 ROUNDS=2 T=300 CMD="python -u bench.py --steps 30 --warmup 5" A="BENCH_SLOTS=2" B="BENCH_SLOTS=3" CUT=200 bash tools/ab.sh && \
ABN=cusplit ROUNDS=2 T=300 CMD="python -u bench.py --steps 30 --warmup 5" A="ATPU_CU_SPLIT=0" B="ATPU_CU_SPLIT=1" CUT=200 bash tools/ab.sh
