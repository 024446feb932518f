# (1) reference-shaped 1-row classify jobs through the agent; (2) GEMM epilogue stagger A/B (item 9);
# (3) persistent-launch prototype: fused T5 FFN block vs two GEMV launches (last: it has a grid barrier)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5i T=300 bash tools/gpu.sh \
  "run:in256f:python -u bench/agent_classify.py --form input --jobs 16384 --max-tasks 256 --controller fast" \
  "run:in256m:python -u bench/agent_classify.py --form input --jobs 8192 --max-tasks 256 --controller mock" \
  "run:in1f:python -u bench/agent_classify.py --form input --jobs 1500 --max-tasks 1 --controller fast" \
  "run:echo256:python -u bench/agent_loop.py --jobs 20000 --max-tasks 256 --controller fast" || exit 1
ABN=stag ROUNDS=2 CMD="python -u bench.py --steps 30 --warmup 5" A="ATPU_NATIVE_PATH=$R/abso/_atpu_stag16.so" B="ATPU_X=0" CUT=110 bash tools/ab.sh || exit 1
ABN=stag40 ROUNDS=2 CMD="python -u bench.py --steps 30 --warmup 5" A="ATPU_NATIVE_PATH=$R/abso/_atpu_stag40.so" B="ATPU_X=0" CUT=110 bash tools/ab.sh || exit 1
OUT=r5i T=180 bash tools/gpu.sh "tests:tests/kernels/test_decode_gpu.py -k t5_ffn_fused" \
  "run:ffn4:python -u tools/bench_ffn_fused.py" "run:ffn1:env ROWS=1 python -u tools/bench_ffn_fused.py"
