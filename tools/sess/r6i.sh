# 1-doc T5 / BART kernel stats after the decode-step work
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r6i T=400 TOPN=30 bash tools/gpu.sh "prof:t5_1doc:bench/summarize.py --docs 1 --steps 3 --warmup 1" \
  "prof:bart_1doc:bench/summarize.py --model bart-large-cnn --docs 1 --steps 3 --warmup 1"
