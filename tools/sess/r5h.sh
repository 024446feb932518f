# persistent-launch prototype: fused T5 FFN block (one in-launch grid barrier) vs two GEMV launches
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5h T=180 bash tools/gpu.sh "tests:tests/kernels/test_decode_gpu.py -k t5_ffn_fused" \
  "run:ffn4:python -u tools/bench_ffn_fused.py" "run:ffn1:env ROWS=1 python -u tools/bench_ffn_fused.py"
