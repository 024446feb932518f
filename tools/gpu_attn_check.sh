#!/bin/bash
# Attention change check on one MI355X: numerics (attention + BERT GPU tests),
# attention microbench, bench.py with the persistent attention on and off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/kernels/test_kernels_gpu.py -k attention tests/kernels/test_bert_gpu.py > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
tail -3 gpurun_out/t_attn.log
timeout -k 10 200 python tools/bench_kernels.py --only attention --rounds 7 > gpurun_out/bk_attn.txt 2>&1 || { tail -20 gpurun_out/bk_attn.txt; exit 1; }
tail -5 gpurun_out/bk_attn.txt
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
ATPU_ATTN_PERSIST=0 timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_p0.json 2>> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json gpurun_out/bench_p0.json
