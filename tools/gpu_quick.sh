#!/bin/bash
# Quick measurement session: C3 bench (default schedule), C3 on the path kernel,
# single-stream frame timeline.  Each GPU step has its own limit; a failure ends it.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/quick
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -c 600 $O/$name.log | tail -2; [ $rc -eq 0 ] || exit $rc; }
step bench_c3 python bench.py --no-cpu --steps 10
step bench_c3_path python bench.py --no-cpu --steps 3 --algo path --no-kernel-times
VARIANTS="split0:RT_TUNE=split=0" bash tools/gpu_timeline.sh
cp gpurun_out/tl_split0.txt $O/ 2>/dev/null
echo done
