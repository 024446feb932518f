# cold load: device random init (tests, bench/cold_load.py with the first-copy H2D probe), bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5b bash tools/gpu.sh "tests:tests/kernels/test_runtime_gpu.py tests/kernels/test_decode_gpu.py -k 'rand_fill or forced_tile or bart_step or cross_split'" \
  "run:cold:python -u bench/cold_load.py --h2d" bench
