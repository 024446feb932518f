# reference-shaped 1-row classify jobs through the agent: 256 per lease and one per lease (MAX_TASKS=1),
# against the asyncio stand-in controller and the test mock; plus the echo loop for the control plane alone
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5g T=400 bash tools/gpu.sh \
  "run:in256f:python -u bench/agent_classify.py --form input --jobs 16384 --max-tasks 256 --controller fast" \
  "run:in256m:python -u bench/agent_classify.py --form input --jobs 8192 --max-tasks 256 --controller mock" \
  "run:in1f:python -u bench/agent_classify.py --form input --jobs 2000 --max-tasks 1 --controller fast" \
  "run:in1m:python -u bench/agent_classify.py --form input --jobs 2000 --max-tasks 1 --controller mock" \
  "run:echo256:python -u bench/agent_loop.py --jobs 20000 --max-tasks 256 --controller fast"
