#!/bin/bash
# PMC passes over the persistent attention kernel (bench_kernels --only attention); one counter group per pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcattn
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_BF16" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmcattn/p$i -o pmc -- python3 $R/tools/bench_kernels.py --only attention --rounds 1 --iters 3 > $R/gpurun_out/pmcattn/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
python3 - <<'PY'
import csv, glob, os, collections
R=os.environ['GRAFT_REPO_ROOT']
agg=collections.defaultdict(list)
for f in sorted(glob.glob(f"{R}/gpurun_out/pmcattn/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if 'attention_packed_persist' not in r.get('Kernel_Name',''): continue
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in sorted(agg.items()):
    print(f"{k:32s} n={len(v):3d} median_per_dispatch={sorted(v)[len(v)//2]:.4g}")
PY
