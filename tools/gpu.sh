#!/bin/bash
# One GPU-box session made of stages, run in order, each under its own time limit; the first
# failing stage ends the session (no retries, nothing after a fault). Logs under gpurun_out/<OUT>/.
#
#   bash tools/gpu.sh tests smoke bench
#   bash tools/gpu.sh "tests:tests/kernels/test_bert_gpu.py -k attention" "bench:--steps 50"
#   bash tools/gpu.sh "run:t5_1024:python -u bench/summarize.py --docs 1024"
#   bash tools/gpu.sh "prof:serial:bench.py --steps 5 --warmup 1"          # rocprofv3 kernel stats
#   bash tools/gpu.sh "pmc:ffn:SQ_WAVES SQ_BUSY_CYCLES:tools/bench_kernels.py --only gemm_ffn1"
#
# Stage forms:
#   tests[:<pytest args>]  GPU tests (default: the whole -m gpu suite); args are eval'd, so quote a -k expression
#   smoke                  __graft_entry__.smoke()
#   bench[:<args>]         bench.py (default --steps 20 --warmup 5)
#   run:<name>:<cmd>       any command; its log is gpurun_out/<OUT>/<name>.log
#   prof:<name>:<script args>   rocprofv3 --kernel-trace --stats of `python3 <script args>`
#   pmc:<name>:<counters>:<script args>  one PMC pass (counters within one block budget)
# Env: OUT (subdir, default "s"), T (per-stage seconds, default 600), STAGE_ENV (extra env for every stage).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/${OUT:-s}
mkdir -p "$O"
T=${T:-600}

summ() {  # per-kernel summary of a rocprofv3 csv stats file
  local f
  f=$(find "$1" -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && python3 "$R/tools/kstats.py" --csv "$f" ${TOPN:-25} > "$1/summary.txt" && cat "$1/summary.txt"
  find "$1" -name '*kernel_trace.csv' -delete 2>/dev/null
  return 0
}

for spec in "$@"; do
  kind=${spec%%:*}
  rest=${spec#*:}
  [ "$rest" = "$spec" ] && rest=""
  echo "[gpu.sh] $(date +%T) stage $spec"
  case $kind in
    tests)
      eval "env $STAGE_ENV timeout -k 10 $T python -u -m pytest -x -v --timeout 120 --timeout-method thread \
        ${rest:--m gpu tests}" > "$O/tests.log" 2>&1
      rc=$?; grep -E "passed|failed|error" "$O/tests.log" | tail -3 ;;
    smoke)
      env $STAGE_ENV timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      rc=$?; tail -2 "$O/smoke.log" ;;
    bench)
      env $STAGE_ENV timeout -k 10 $T python -u bench.py ${rest:---steps 20 --warmup 5} > "$O/bench.log" 2>&1
      rc=$?; grep -v amdgpu.ids "$O/bench.log" | tail -2 | cut -c1-600 ;;
    run)
      name=${rest%%:*}; cmd=${rest#*:}
      env $STAGE_ENV timeout -k 10 $T $cmd > "$O/$name.log" 2>&1
      rc=$?; grep -v amdgpu.ids "$O/$name.log" | tail -${TAILN:-3} | cut -c1-600 ;;
    prof)
      name=${rest%%:*}; cmd=${rest#*:}
      (cd /tmp && export TMPDIR=/tmp && env $STAGE_ENV timeout -k 10 $T rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$O/$name" -o run -- python3 $R/$cmd > "$O/$name.log" 2>&1)
      rc=$?; grep -v amdgpu.ids "$O/$name.log" | tail -1 | cut -c1-400; [ $rc -eq 0 ] && summ "$O/$name" ;;
    pmc)
      name=${rest%%:*}; rest2=${rest#*:}; ctr=${rest2%%:*}; cmd=${rest2#*:}
      (cd /tmp && export TMPDIR=/tmp && env $STAGE_ENV timeout -s KILL 120 rocprofv3 --pmc $ctr \
        --output-format csv -d "$O/$name" -o pmc -- python3 $R/$cmd > "$O/$name.log" 2>&1)
      rc=$?; tail -1 "$O/$name.log" ;;
    *) echo "unknown stage $spec"; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "[gpu.sh] stage '$spec' failed rc=$rc"; exit $rc
  fi
done
echo "[gpu.sh] $(date +%T) all stages ok"
