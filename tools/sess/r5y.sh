# round-5 numbers for the README table: 1-doc and 1024-doc summarize, 1-doc agent jobs
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5y T=400 bash tools/gpu.sh "run:t5_1doc:python -u bench/summarize.py --docs 1 --steps 20 --warmup 3" \
  "run:bart_1doc:python -u bench/summarize.py --model bart-large-cnn --docs 1 --steps 20 --warmup 3" \
  "run:t5_1024:python -u bench/summarize.py --docs 1024 --steps 2" \
  "run:agent_t5_1doc:python -u bench/agent_summarize.py --max-tasks 1 --batch 0 --jobs 200" \
  "run:agent_bart_1doc:python -u bench/agent_summarize.py --model bart-large-cnn --max-tasks 1 --batch 0 --jobs 200"
