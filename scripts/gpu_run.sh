#!/bin/bash
# One parametrised GPU session (replaces the round-2 one-off gpu_r2*.sh files).
# Every step runs under its own time limit.  The script stops at the first
# failing step -- no GPU step runs after a fault, abort or time-out -- except a
# pytest step whose tests merely failed (exit 1: assertions, no crash), after
# which the next steps still run; the script then exits 1 at the end.
#
# usage (on the box, from the repo root):
#   scripts/gpu_run.sh TAG STEP [STEP ...]
# steps:
#   pytest:<files or -k expression, comma separated>   e.g. pytest:tests/test_gpu_kkt.py,tests/test_gpu_admm.py
#   pytest-all                                           the whole -m gpu suite
#   py:<script args, comma separated>                    e.g. py:scripts/prof_c5.py
#   trace:<script args, comma separated>                 rocprofv3 --kernel-trace --stats of that script
#   rtrace:<script args, comma separated>                the same plus the HIP runtime API trace (host-side call times)
#   bench:<bench.py args, comma separated>               e.g. bench:--no-cpu,--steps,20
#   lat                                                  scripts/ubench/lat_bench
#   pmc:<tag>,<dominant kernel>,<script args...>         PMC passes of one workload (scripts/collect_pmc.sh)
#   env:NAME=VALUE / unenv:NAME                          set / clear an environment variable for the later steps
#                                                        (A/B of a variant library: env:PDPLQR_LIB=<path>)
# outputs: gpurun_out/TAG/<step index>_<kind>.{log,json}, trace dirs under gpurun_out/TAG/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  args=${arg//,/ }
  log=$O/${i}_${kind}.log
  echo "== step $i: $kind $args" | tee -a "$O/steps.log"
  case $kind in
    pytest)
      timeout -k 10 900 python -u -m pytest $args -m gpu -x -v --timeout 300 --timeout-method thread > "$log" 2>&1 ;;
    pytest-all)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$log" 2>&1 ;;
    py)
      timeout -k 10 600 python -u $args > "$log" 2>&1 ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$i" -o run -- python -u $args > "$log" 2>&1 ;;
    rtrace)
      timeout -k 10 600 rocprofv3 --runtime-trace --kernel-trace --stats --output-format csv -d "$O/rtrace_$i" -o run -- python -u $args > "$log" 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py $args > "$log" 2>&1 ;;
    lat)
      timeout -k 10 60 ./scripts/ubench/lat_bench > "$log" 2>&1 ;;
    pmc)
      set -- $args
      ptag=$1; pdom=$2; shift 2
      TAG=$ptag DOM=$pdom OUT=$O/pmc_$ptag timeout -k 10 1200 scripts/collect_pmc.sh python3 "$@" > "$log" 2>&1 ;;
    env)
      export "$arg"; echo "rc=0" >> "$O/steps.log"; continue ;;
    unenv)
      unset "$arg"; echo "rc=0" >> "$O/steps.log"; continue ;;
    *)
      echo "unknown step $kind" | tee -a "$O/steps.log"; exit 2 ;;
  esac
  rc=$?
  tail -3 "$log" | tee -a "$O/steps.log"
  echo "rc=$rc" | tee -a "$O/steps.log"
  if [ $rc -eq 1 ] && { [ "$kind" = pytest ] || [ "$kind" = pytest-all ]; }; then
    failed=1
    continue
  fi
  [ $rc -eq 0 ] || exit $rc
done
exit ${failed:-0}
