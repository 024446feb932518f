# BART-large-CNN 256-doc summarize kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r6j T=400 TOPN=30 bash tools/gpu.sh "prof:bart_256:bench/summarize.py --model bart-large-cnn --docs 256 --steps 1 --warmup 1"
