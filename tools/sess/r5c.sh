# cold load (warm-process LRU misses, first-copy probe), summarize stage clocks, encoder kernel sum
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5c bash tools/gpu.sh "run:cold:python -u bench/cold_load.py --h2d" \
  "run:enc:python -u tools/check_encode_timing.py" \
  "prof:encprof:tools/check_encode_timing.py --encode-only --reps 4" \
  "run:s256:python -u bench/summarize.py --docs 256 --steps 2" \
  "run:b256:python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2"
