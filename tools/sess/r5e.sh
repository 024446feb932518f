# 8-rank rehearsals on one GPU (gloo; ranks share the card): bench self-launch, bench under an
# external torch.distributed.run, the DP=8 agent classify job; summarize encode clock re-check
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
export TORCH_NCCL_ASYNC_ERROR_HANDLING=1
OUT=r5e T=420 bash tools/gpu.sh \
  "run:b8self:python -u bench.py --gpus 8 --dist-backend gloo --steps 5 --warmup 2 --batch-rows 512" \
  "run:b8ext:python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 8 --dist-backend gloo --steps 5 --warmup 2 --batch-rows 512" \
  "run:agent8:python -u bench/agent_classify.py --jobs 8 --shard 8192 --output summary --dp 8 --dp-backend gloo" \
  "run:enc:python -u tools/check_encode_timing.py --reps 2"
