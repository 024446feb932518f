#!/bin/bash
# Headline bench (BERT-base), BERT-large bench, rocprofv3 kernel stats (serial + concurrent) of the headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/refresh
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/refresh/base.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --model bert-large --batch-rows 512 --steps 10 --warmup 3 > gpurun_out/refresh/large.log 2>&1 || exit $?
grep -h metric gpurun_out/refresh/base.log gpurun_out/refresh/large.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp
ATPU_CONCURRENT_SLOTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/refresh/serial -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/refresh/serial.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/refresh/conc -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/refresh/conc.log 2>&1 || exit $?
ls $R/gpurun_out/refresh/serial $R/gpurun_out/refresh/conc
