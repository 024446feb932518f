# long-K decode GEMMs: forced split-K counts
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5w
timeout -k 10 300 python -u tools/bench_dec_splitk.py > gpurun_out/r5w/splitk.jsonl 2>&1; rc=$?
cat gpurun_out/r5w/splitk.jsonl; exit $rc
