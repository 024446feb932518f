# host-side split of the 1-doc decode step (is the GPU ever waiting for the host?)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6n
timeout -k 10 200 python -u tools/host_prof_summ.py t5-base 1 > gpurun_out/r6n/t5.log 2>&1 && timeout -k 10 200 python -u tools/host_prof_summ.py bart-large-cnn 1 > gpurun_out/r6n/bart.log 2>&1; rc=$?
grep -h docs= gpurun_out/r6n/*.log; exit $rc
