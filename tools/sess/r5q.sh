# validation after the tokenizer rewrite: full GPU suite, smoke, headline bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5q bash tools/gpu.sh tests smoke bench
