set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model bert-large --steps 10 --warmup 2 > gpurun_out/b_large.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/b_large.json
