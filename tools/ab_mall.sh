#!/bin/bash
# Cache-policy x batch-size sweep of the headline bench: do smaller per-step batches with
# default-policy (L2/MALL-allocating) stores keep a layer's activations in the 256 MB
# Infinity Cache? Each config: "rows gemm256 attn_nt slots". Interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/abmall
CONFIGS=${CONFIGS:-"1024 n 1 2|256 n 1 2|256 l 0 2|512 l 0 2|256 l 0 1|128 l 0 2|1024 l 0 2"}
IFS='|' read -ra CF <<< "$CONFIGS"
for r in 1 2; do
  for c in "${CF[@]}"; do
    read -r b g nt sl <<< "$c"
    tag="b${b}_g${g}_nt${nt}_s${sl}_r${r}"
    ATPU_GEMM_256=$g ATPU_ATTN_NT=$nt timeout -k 10 300 python -u bench.py --batch-rows $b --slots $sl \
      --steps $((20480 / b)) --warmup 4 > gpurun_out/abmall/$tag.log 2>&1 || exit $?
    echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/abmall/$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abmall/$tag.log)"
  done
done
