# ws kernel cycle stamps (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5m
ATPU_NATIVE_PATH=$GRAFT_REPO_ROOT/abso/_atpu_stamps.so timeout -k 10 300 python -u tools/ws_stamps.py --variants 0,8 > gpurun_out/r5m/stamps.jsonl 2>&1; rc=$?
cat gpurun_out/r5m/stamps.jsonl; exit $rc
