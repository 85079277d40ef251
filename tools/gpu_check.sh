#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() { # pytest returns 1 for failed assertions; anything else >1 is fatal here
  local rc=$1 what=$2
  echo "$what rc=$rc"
  if [ "$rc" -gt 1 ]; then echo "fatal exit from $what, stopping"; exit "$rc"; fi
}
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rA ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
stop_if_fatal $? pytest
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
stop_if_fatal $? smoke
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
stop_if_fatal $? bench
tail -1 gpurun_out/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py ${BENCH_ARGS:-} --no-cpu > gpurun_out/prof.log 2>&1
  stop_if_fatal $? rocprof
  find gpurun_out/prof -name "*stats*" | head
fi
if [ "${PMC:-1}" = "1" ]; then
  GROUPS_PMC="FETCH_SIZE;WRITE_SIZE" BENCH_ARGS="${BENCH_ARGS:-} --no-cpu" bash tools/gpu_pmc.sh
  stop_if_fatal $? pmc
fi
