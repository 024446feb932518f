#!/bin/bash
# Round-end evidence: headline + BERT-large benches, summarize benches, rocprofv3 kernel stats
# (headline serial / concurrent, T5 and BART summarize). Every GPU step time-limited, && chained.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/base.log 2>&1 && echo "base done" \
 && timeout -k 10 400 python -u bench.py --model bert-large --batch-rows 512 --steps 10 --warmup 3 > $O/large.log 2>&1 && echo "large done" \
 && timeout -k 10 300 python -u bench/summarize.py --docs 256 > $O/t5_256.log 2>&1 && echo "t5 256 done" \
 && timeout -k 10 400 python -u bench/summarize.py --docs 1024 > $O/t5_1024.log 2>&1 && echo "t5 1024 done" \
 && timeout -k 10 300 python -u bench/summarize.py --docs 256 --model bart-large-cnn > $O/bart_256.log 2>&1 && echo "bart done" \
 && cd /tmp && export TMPDIR=/tmp \
 && ATPU_CONCURRENT_SLOTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $O/serial.log 2>&1 && echo "serial prof done" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/conc -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $O/conc.log 2>&1 && echo "conc prof done" \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t5 -o run -- python3 $R/bench/summarize.py --docs 256 --steps 1 --warmup 1 > $O/t5prof.log 2>&1 && echo "t5 prof done" \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bart -o run -- python3 $R/bench/summarize.py --docs 256 --steps 1 --warmup 1 --model bart-large-cnn > $O/bartprof.log 2>&1 && echo "bart prof done"
rc=$?
cd $R
grep -h metric $O/*.log | cut -c1-200
find $O -name '*kernel_trace.csv' -delete
exit $rc
