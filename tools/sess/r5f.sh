# GELU without the input clamp: is the cross-pipeline test's margin the weights or the GELU (base build);
# accuracy / LN-fold / headline tests; bench A/B vs the base build
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5f STAGE_ENV="ATPU_NATIVE_PATH=$R/abso/_atpu_base.so" bash tools/gpu.sh "tests:tests/kernels/test_bert_gpu.py -k production_batch" ; echo "base-build production test rc=$?"
OUT=r5f bash tools/gpu.sh "tests:tests/kernels/test_kernels_gpu.py tests/kernels/test_ln_fold_gpu.py tests/kernels/test_headline_gpu.py tests/kernels/test_bert_gpu.py" || exit 1
ABN=gelu ROUNDS=3 CMD="python -u bench.py --steps 30 --warmup 5" A="ATPU_NATIVE_PATH=$R/abso/_atpu_base.so" B="ATPU_X=1" CUT=120 bash tools/ab.sh
