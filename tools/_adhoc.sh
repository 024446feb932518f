set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
rm -rf gpurun_out/prof_serial gpurun_out/prof_conc
mkdir -p gpurun_out/prof_serial gpurun_out/prof_conc
cd /tmp && export TMPDIR=/tmp
ATPU_CONCURRENT_SLOTS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $R/gpurun_out/prof_serial -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/prof_serial.log 2>&1 || { tail -30 $R/gpurun_out/prof_serial.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $R/gpurun_out/prof_conc -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/prof_conc.log 2>&1 || { tail -30 $R/gpurun_out/prof_conc.log; exit 1; }
cd $R
for d in prof_serial prof_conc; do f=$(find gpurun_out/$d -name '*.db' | head -1); (python tools/kstats.py $f 16 > gpurun_out/$d.txt && head -8 gpurun_out/$d.txt) || find gpurun_out/$d; done
