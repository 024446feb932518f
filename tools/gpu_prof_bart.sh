#!/bin/bash
# rocprofv3 kernel stats of the BART-large-CNN summarize bench (256 docs, one step).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bartprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 $R/bench/summarize.py --docs 256 --steps 1 --warmup 1 --model bart-large-cnn > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
exit $rc
