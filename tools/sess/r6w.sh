# round-5 end state: full GPU suite, smoke, headline bench, serial kernel profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r6w bash tools/gpu.sh tests smoke bench && OUT=r6w STAGE_ENV="ATPU_CONCURRENT_SLOTS=0" bash tools/gpu.sh "prof:serial:bench.py --steps 5 --warmup 1"
