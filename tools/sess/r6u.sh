# summarize part split default 128: 512-doc A/B (one search vs 3 parts), 256-doc T5 / BART with the new default
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=parts512_t5 ROUNDS=1 T=500 CMD="python -u bench/summarize.py --docs 512 --steps 1" A="ATPU_SUMM_PART_MIN=300" B="ATPU_SUMM_PART_MIN=128" CUT=200 bash tools/ab.sh && \
OUT=r6u T=400 bash tools/gpu.sh "run:t5_256:python -u bench/summarize.py --docs 256 --steps 2" "run:bart_256:python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2" "run:t5_1024:python -u bench/summarize.py --docs 1024 --steps 1"
