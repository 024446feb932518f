# few-row LM head kernel: lm_head + decode tests, per-call time, T5 / BART 1-doc A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6e
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu > gpurun_out/r6e/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6e/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_lm_few.py --rounds 3 > gpurun_out/r6e/lm_few.jsonl 2>&1 && ATPU_AB_LM_FEW=0 timeout -k 10 300 python -u tools/bench_lm_few.py --rounds 3 > gpurun_out/r6e/lm_old.jsonl 2>&1; rc=$?
grep -v amdgpu gpurun_out/r6e/lm_few.jsonl gpurun_out/r6e/lm_old.jsonl; [ $rc -eq 0 ] || exit $rc
ABN=lmfew_t5 ROUNDS=3 T=300 CMD="python -u bench/summarize.py --docs 1 --steps 20 --warmup 3" A="ATPU_AB_LM_FEW=0" B="ATPU_AB_LM_FEW=1" CUT=250 bash tools/ab.sh && \
ABN=lmfew_bart ROUNDS=3 T=300 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 1 --steps 20 --warmup 3" A="ATPU_AB_LM_FEW=0" B="ATPU_AB_LM_FEW=1" CUT=250 bash tools/ab.sh
