# dec kernel: 2 K-tiles per barrier A/B (decode shapes)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5r
timeout -k 10 300 python -u tools/bench_dec_kpb.py --rows 1024,256 > gpurun_out/r5r/kpb.jsonl 2>&1; rc=$?
cat gpurun_out/r5r/kpb.jsonl; exit $rc
