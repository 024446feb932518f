# round-5 baseline after the negative-path cleanup: GPU tests, headline bench, serial kernel profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5a bash tools/gpu.sh bench "tests" && OUT=r5a STAGE_ENV="ATPU_CONCURRENT_SLOTS=0" bash tools/gpu.sh "prof:serial:bench.py --steps 5 --warmup 1"
