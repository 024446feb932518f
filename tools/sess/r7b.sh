# 256-doc summarize (2 parts of 512 rows): decode GEMM split-K heuristic vs never split
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=nosplit_t5 ROUNDS=2 T=400 CMD="python -u bench/summarize.py --docs 256 --steps 2" A="ATPU_GEMM_SPLITK=-1" B="ATPU_GEMM_SPLITK=1" CUT=200 bash tools/ab.sh && \
ABN=nosplit_bart ROUNDS=2 T=400 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2" A="ATPU_GEMM_SPLITK=-1" B="ATPU_GEMM_SPLITK=1" CUT=200 bash tools/ab.sh
