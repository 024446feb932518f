set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/kernels/test_decode_gpu.py -x -q > gpurun_out/pytest_dec.log 2>&1 || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -2 gpurun_out/pytest_dec.log
timeout -k 10 500 python bench/summarize.py --model bart-large-cnn --docs 64 --steps 2 --warmup 1 > gpurun_out/summ_bart64.log 2>&1 || { tail -30 gpurun_out/summ_bart64.log; exit 1; }
tail -1 gpurun_out/summ_bart64.log
timeout -k 10 500 python bench/summarize.py --model bart-large-cnn --docs 256 --steps 1 --warmup 1 > gpurun_out/summ_bart256.log 2>&1 || { tail -30 gpurun_out/summ_bart256.log; exit 1; }
tail -1 gpurun_out/summ_bart256.log
