# headline: plain stores for the hidden-state outputs (o-proj / FFN2, read next by FFN1 / QKV), non-temporal for FFN1's
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=plainx ROUNDS=3 T=300 CMD="python -u bench.py --steps 30 --warmup 5" A="ATPU_GEMM_PLAIN_X=0" B="ATPU_GEMM_PLAIN_X=1" CUT=200 bash tools/ab.sh
