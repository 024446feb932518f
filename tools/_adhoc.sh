set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "gemm" tests/kernels/test_bert_gpu.py > gpurun_out/t_res.log 2>&1 || { tail -30 gpurun_out/t_res.log; exit 1; }
tail -2 gpurun_out/t_res.log
timeout -k 10 200 python tools/bench_kernels.py --only gemm_o_res,gemm_ffn2_res,gemm_qkv --rounds 7 > gpurun_out/bk_res.txt 2>&1 || { tail -20 gpurun_out/bk_res.txt; exit 1; }
grep -v JSON gpurun_out/bk_res.txt | tail -3
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
