#!/bin/bash
# Summarize end to end after the host-side tokenize / word-map rework: T5 and BART at 256 docs,
# T5 at 1024 docs, plus the host-side split of a decode step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/summhost
mkdir -p $O
timeout -k 10 300 python -u bench/summarize.py --docs 256 > $O/t5_256.log 2>&1 && echo "t5 256 $(grep -o '"value": [0-9.]*' $O/t5_256.log)" \
 && timeout -k 10 300 python -u bench/summarize.py --docs 256 --model bart-large-cnn > $O/bart_256.log 2>&1 && echo "bart 256 $(grep -o '"value": [0-9.]*' $O/bart_256.log)" \
 && timeout -k 10 400 python -u bench/summarize.py --docs 1024 > $O/t5_1024.log 2>&1 && echo "t5 1024 $(grep -o '"value": [0-9.]*' $O/t5_1024.log)" \
 && timeout -k 10 300 python -u tools/host_prof_summ.py t5-base 256 > $O/hostprof_t5.log 2>&1 && tail -n 1 $O/hostprof_t5.log
