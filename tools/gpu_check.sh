#!/bin/bash
# One GPU round-trip: kernel/model tests, smoke, headline bench. Each step time-limited, chained with &&.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log; tail -2 gpurun_out/smoke.log; tail -2 gpurun_out/bench.log
exit $rc
