# encoder GEMMs on real activations vs random of the same statistics
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5p
timeout -k 10 400 python -u tools/bench_gemm_realdata.py > gpurun_out/r5p/realdata.jsonl 2>&1; rc=$?
cat gpurun_out/r5p/realdata.jsonl | tail -12; exit $rc
