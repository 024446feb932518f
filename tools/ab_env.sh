#!/bin/bash
# A/B one environment toggle in alternating processes. Usage:
#   CMD="python bench/summarize.py --docs 256" A="ATPU_RMS_FOLD=0" B="ATPU_RMS_FOLD=1" ROUNDS=2 bash tools/ab_env.sh
set -o pipefail
mkdir -p gpurun_out/abenv
for r in $(seq 1 ${ROUNDS:-2}); do
  for side in A B; do
    env ${!side} timeout -k 10 300 $CMD > gpurun_out/abenv/${side}_r$r.log 2>&1 || exit $?
    echo "round $r $side (${!side}): $(grep -v amdgpu.ids gpurun_out/abenv/${side}_r$r.log | grep -v '^JSON' | tail -${TAILN:-1} | cut -c1-${CUT:-200})"
  done
done
