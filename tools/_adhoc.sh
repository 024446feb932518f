set -o pipefail
mkdir -p gpurun_out
for split in 0 1 0 1; do
  ATPU_CU_SPLIT=$split timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_s$split.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_s$split.json'));print('split',$split,d['value'],d['ms_per_step'],d['config']['cu_split'])"
done
