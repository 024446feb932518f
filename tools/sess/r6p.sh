# dev build (ws kernels, LM-head configs, timing ablations): its GPU tests, incl. the dev-only ones
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6p
ATPU_NATIVE_PATH=$R/abso/_atpu_dev.so timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/kernels/test_qkv_attention_gpu.py tests/kernels/test_gemm_ws_gpu.py tests/kernels/test_decode_gpu.py -k "ws or lm_head or qkv" > gpurun_out/r6p/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6p/tests.log; exit $rc
