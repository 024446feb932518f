#!/bin/bash
# A/B two configurations of one command in alternating processes (ROUNDS rounds).
#   env toggle:  CMD="python bench.py --steps 20" A="ATPU_X=0" B="ATPU_X=1" bash tools/ab.sh
#   two builds:  CMD="python tools/bench_kernels.py --only attention" A="ATPU_NATIVE_PATH=$PWD/abso/_atpu_base.so" B="" bash tools/ab.sh
# Every run is time-limited; the first failure ends the session. Prints the last TAILN lines of each run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/ab${ABN:-}
mkdir -p "$O"
for r in $(seq 1 ${ROUNDS:-2}); do
  for side in A B; do
    env ${!side} timeout -k 10 ${T:-300} $CMD > "$O/${side}_r$r.log" 2>&1 || { tail -5 "$O/${side}_r$r.log"; exit 1; }
    echo "round $r $side (${!side}): $(grep -v amdgpu.ids "$O/${side}_r$r.log" | tail -${TAILN:-1} | cut -c1-${CUT:-300})"
  done
done
