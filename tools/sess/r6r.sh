# BERT-large serial kernel profile (1024 rows)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r6r STAGE_ENV="ATPU_CONCURRENT_SLOTS=0" TOPN=20 bash tools/gpu.sh "prof:large:bench.py --model bert-large --steps 3 --warmup 1"
