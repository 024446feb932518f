# flash encoder attention: fewer VALU per score (bias base + immediates, FMA, MFMA row sums); tests, then A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5s
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_kernels_gpu.py tests/kernels/test_decode_gpu.py -m gpu -k "flash or dist_bias or long_source" > gpurun_out/r5s/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5s/tests.log
[ $rc -eq 0 ] || exit $rc
ABN=flash ROUNDS=3 TAILN=2 CUT=200 CMD="python -u tools/bench_kernels.py --only attn_flash_t5,attn_flash_bart --rounds 3" A="ATPU_NATIVE_PATH=$R/abso/_atpu_base.so" B="ATPU_X=0" bash tools/ab.sh
