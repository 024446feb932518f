# round-5 close: full GPU suite, smoke, headline bench; then agent 1-doc summarize jobs batched per lease
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r7a bash tools/gpu.sh tests smoke bench && \
OUT=r7a T=500 bash tools/gpu.sh "run:agent_t5_256:python -u bench/agent_summarize.py --jobs 1024 --max-tasks 256" \
  "run:agent_t5_1024:python -u bench/agent_summarize.py --jobs 2048 --max-tasks 1024" \
  "run:agent_bart_256:python -u bench/agent_summarize.py --model bart-large-cnn --jobs 1024 --max-tasks 256"
