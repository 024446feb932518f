# dec kernel two K groups: decode tests with KG=2, per-shape A/B, T5 + BART summarize A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5x
ATPU_DEC_KG=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_gpu.py -m gpu --deselect "tests/kernels/test_decode_gpu.py::test_engine_stream_split_matches_single" > gpurun_out/r5x/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5x/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_dec_kg.py > gpurun_out/r5x/kg.jsonl 2>&1; rc=$?
cat gpurun_out/r5x/kg.jsonl
[ $rc -eq 0 ] || exit $rc
ABN=kg_t5 ROUNDS=2 T=400 CMD="python -u bench/summarize.py --docs 256 --steps 2" A="ATPU_DEC_KG=1" B="ATPU_DEC_KG=2" bash tools/ab.sh && \
ABN=kg_bart ROUNDS=2 T=400 CMD="python -u bench/summarize.py --model bart-large-cnn --docs 256 --steps 2" A="ATPU_DEC_KG=1" B="ATPU_DEC_KG=2" bash tools/ab.sh
