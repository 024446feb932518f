# LM head at few rows: per-config call time (release + dev build), T5 1-doc kernel stats with the few-row merge
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6d
timeout -k 10 300 python -u tools/bench_lm_few.py > gpurun_out/r6d/lm_rel.jsonl 2>&1; rc=$?; cat gpurun_out/r6d/lm_rel.jsonl | grep -v amdgpu; [ $rc -eq 0 ] || exit $rc
ATPU_NATIVE_PATH=$R/abso/_atpu_dev.so timeout -k 10 300 python -u tools/bench_lm_few.py > gpurun_out/r6d/lm_dev.jsonl 2>&1; rc=$?; cat gpurun_out/r6d/lm_dev.jsonl | grep -v amdgpu; [ $rc -eq 0 ] || exit $rc
OUT=r6d T=400 TOPN=20 bash tools/gpu.sh "prof:t5_1doc:bench/summarize.py --docs 1 --steps 3 --warmup 1"
