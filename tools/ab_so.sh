#!/bin/bash
# A/B two builds of the extension in alternating processes: base = abso/_atpu_base.so, new = in-tree build.
# Usage: CMD="python tools/bench_kernels.py --only attention" ROUNDS=3 bash tools/ab_so.sh
set -o pipefail
mkdir -p gpurun_out/abso
for r in $(seq 1 ${ROUNDS:-2}); do
  ATPU_NATIVE_PATH=$PWD/abso/_atpu_base.so timeout -k 10 300 $CMD > gpurun_out/abso/base_r$r.log 2>&1 || exit $?
  timeout -k 10 300 $CMD > gpurun_out/abso/new_r$r.log 2>&1 || exit $?
  echo "round $r base: $(grep -v amdgpu.ids gpurun_out/abso/base_r$r.log | grep -v '^JSON' | tail -${TAILN:-1} | cut -c1-${CUT:-200})"
  echo "round $r new : $(grep -v amdgpu.ids gpurun_out/abso/new_r$r.log | grep -v '^JSON' | tail -${TAILN:-1} | cut -c1-${CUT:-200})"
done
