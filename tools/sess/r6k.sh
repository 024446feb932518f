# probe: few workgroups streaming a head's QKV slice each
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6k
timeout -k 10 60 ./tools/probes/few_cu_stream > gpurun_out/r6k/stream.jsonl 2>&1; rc=$?; cat gpurun_out/r6k/stream.jsonl; exit $rc
