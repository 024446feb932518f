set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
mkdir -p gpurun_out/prof_bench gpurun_out/prof_t5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/prof_bench.log 2>&1 || { tail -30 $R/gpurun_out/prof_bench.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $R/gpurun_out/prof_t5 -o run -- python3 $R/bench/summarize.py --model t5-base --docs 256 --steps 1 --warmup 1 > $R/gpurun_out/prof_t5.log 2>&1 || { tail -30 $R/gpurun_out/prof_t5.log; exit 1; }
cd $R
for d in prof_bench prof_t5; do f=$(find gpurun_out/$d -name '*.db' | head -1); (python tools/kstats.py $f 22 > gpurun_out/$d.txt && cat gpurun_out/$d.txt) || find gpurun_out/$d; done
