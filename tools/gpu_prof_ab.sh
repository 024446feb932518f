#!/bin/bash
# rocprofv3 kernel stats of the serial bench (ATPU_CONCURRENT_SLOTS=0) under two env settings: A=$PROF_A, B=$PROF_B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/profab
cd /tmp && export TMPDIR=/tmp
for tag in A B; do
  envs=$([ $tag = A ] && echo "${PROF_A:-}" || echo "${PROF_B:-}")
  env ATPU_CONCURRENT_SLOTS=0 $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profab/$tag -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/profab/$tag.log 2>&1 || exit $?
done
for tag in A B; do
  f=$(find $R/gpurun_out/profab/$tag -name '*kernel_stats.csv' | head -1)
  echo "== $tag ($([ $tag = A ] && echo "${PROF_A:-default}" || echo "${PROF_B:-default}")): $f"
  python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.2f} ms")
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):5d} x {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:110]}")
PY
done
