# MI355X (gfx950) agent image. Base: ROCm 7.x + PyTorch-ROCm (provides torch, RCCL, hipcc).
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

ENV PYTHONUNBUFFERED=1 \
    PYTHONDONTWRITEBYTECODE=1 \
    PIP_DISABLE_PIP_VERSION_CHECK=1 \
    PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0

WORKDIR /app
COPY requirements.txt /app/requirements.txt
RUN pip install --no-cache-dir requests psutil pybind11

COPY . /app
# compile every HIP/C++ source for gfx950 in-tree (no GPU needed at build time)
RUN python agent_tpu_amd/csrc/build.py --force

ENV CONTROLLER_URL=http://controller:8080 \
    AGENT_NAME=agent-mi355x-base \
    TASKS=echo,map_classify,map_classify_tpu,risk_accumulate,read_csv_shard,map_tokenize,map_summarize

# single GPU: python app.py ; whole node (one rank per GPU):
#   torchrun --nproc-per-node 8 --master-addr 127.0.0.1 app.py
CMD ["python", "app.py"]
