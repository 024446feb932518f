# Developer entry points. GPU targets need an MI355X (use gpurun on the dev pool).
PY ?= python
NPROC ?= 8

.PHONY: build build-debug test test-gpu test-gpu-serial test-dist sanitize bench bench-dp bench-summarize bench-risk bench-agent profile clean

build:            ## compile every HIP/C++ source for gfx950 in-tree
	$(PY) agent_tpu_amd/csrc/build.py

build-debug:
	$(PY) agent_tpu_amd/csrc/build.py --force --debug

test: build       ## CPU suite: contracts, HF parity, integration, gloo DP, host sanitizers
	$(PY) -m pytest tests -m "not gpu" -q

test-gpu: build   ## kernel numerics + model/op tests on the GPU
	$(PY) -m pytest tests -m gpu -q

test-gpu-serial: build  ## same, every launch synchronous + serialized (localises a faulting kernel)
	HIP_LAUNCH_BLOCKING=1 AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 $(PY) -m pytest tests -m gpu -q -x

test-dist:
	$(PY) -m pytest tests/distributed -q

sanitize:         ## host C++ (CSV index, tokenizer) under ASan + UBSan
	$(PY) -m pytest tests/contract/test_host_sanitizers.py -q

bench:            ## headline: classified rows/s, BERT-base, 1 GPU
	$(PY) bench.py

bench-dp:         ## whole node, one rank per GPU over RCCL
	$(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $(NPROC) --master-addr 127.0.0.1 \
	  --master-port 29555 bench.py --gpus $(NPROC)

bench-summarize:
	$(PY) bench/summarize.py --docs 256
	$(PY) bench/summarize.py --model bart-large-cnn --docs 256

bench-risk:
	$(PY) bench/risk_scaling.py

bench-agent:
	$(PY) bench/agent_loop.py

profile:          ## per-kernel stats of the headline bench (run from any dir; TMPDIR=/tmp)
	cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats -d $(CURDIR)/gpurun_out/prof -o bench -- \
	  $(PY) $(CURDIR)/bench.py --steps 5 --warmup 2

clean:
	rm -rf build agent_tpu_amd/_atpu*.so
