# validation after the decode-step work: full GPU suite, smoke, headline bench, 1-doc + 256-doc summarize
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r6v bash tools/gpu.sh tests smoke bench "run:t5_1doc:python -u bench/summarize.py --docs 1 --steps 20 --warmup 3" \
  "run:bart_1doc:python -u bench/summarize.py --model bart-large-cnn --docs 1 --steps 20 --warmup 3" \
  "run:t5_256:python -u bench/summarize.py --docs 256 --steps 2" \
  "run:agent_t5_1doc:python -u bench/agent_summarize.py --max-tasks 1 --batch 0 --jobs 200" \
  "run:agent_bart_1doc:python -u bench/agent_summarize.py --model bart-large-cnn --max-tasks 1 --batch 0 --jobs 200"
