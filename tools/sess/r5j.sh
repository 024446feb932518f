# checkpoint validation of the committed tree: full GPU suite, smoke, headline bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5j bash tools/gpu.sh tests smoke bench
