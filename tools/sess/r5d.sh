# GPU: new tests (rand init, engine memory vs sizing), bert-large batch A/B, agent cold first job,
# encoder kernels under a generate() profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OUT=r5d bash tools/gpu.sh "tests:tests/kernels/test_runtime_gpu.py -k 'rand_fill or row_bytes'" \
  "run:large1024:python -u bench.py --model bert-large --steps 10 --warmup 3" \
  "run:large512:python -u bench.py --model bert-large --batch-rows 512 --steps 10 --warmup 3" \
  "run:large1024b:python -u bench.py --model bert-large --steps 10 --warmup 3" \
  "run:agent:python -u bench/agent_classify.py --jobs 8 --output summary" \
  "prof:genprof:tools/check_encode_timing.py --reps 2"
