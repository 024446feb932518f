#!/bin/bash
# rocprofv3 kernel stats of the T5-base summarize bench (256 docs, 1 step).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/profsumm
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profsumm -o run -- python3 $R/bench/summarize.py --docs ${DOCS:-256} --steps 1 --warmup 1 > $R/gpurun_out/profsumm/log.txt 2>&1 || exit $?
f=$(find $R/gpurun_out/profsumm -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:100]}")
PY
