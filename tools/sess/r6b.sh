# GEMM output store policy end to end: non-temporal (default 256n) vs plain (256l)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=ntst ROUNDS=3 T=300 CMD="python -u bench.py --steps 30 --warmup 5" A="ATPU_GEMM_256=n" B="ATPU_GEMM_256=l" CUT=200 bash tools/ab.sh
