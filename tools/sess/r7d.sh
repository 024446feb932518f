# round-5 final: full GPU suite, smoke, headline bench, serial kernel profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r7d bash tools/gpu.sh tests smoke bench && OUT=r7d STAGE_ENV="ATPU_CONCURRENT_SLOTS=0" bash tools/gpu.sh "prof:serial:bench.py --steps 5 --warmup 1"
