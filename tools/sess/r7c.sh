# dec-kernel split-K threshold 128 -> 64 blocks: decode tests, 256-doc T5 / BART
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r7c
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py tests/kernels/test_kernels_gpu.py -m gpu > gpurun_out/r7c/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r7c/tests.log
[ $rc -eq 0 ] || exit $rc
OUT=r7c T=400 bash tools/gpu.sh "run:t5_256:python -u bench/summarize.py --docs 256 --steps 2" "run:bart_256:python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2" "run:t5_1024:python -u bench/summarize.py --docs 1024 --steps 1"
