#!/bin/bash
# Exploration session: default vs single-stream frame timelines (kernel-alone
# durations), the per-pixel path kernel at C3, and the C4 / C5 bench lines.
# Each GPU step has its own limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/explore
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
VARIANTS="${TL_VARIANTS:-default:X=1 single:RT_TUNE=split=0}" bash tools/gpu_timeline.sh || exit $?
step bench_path_c3 300 python bench.py --algo path --no-cpu --no-gather --no-kernel-times
step bench_c4 400 python bench.py --config c4
step bench_c5 600 python bench.py --config c5 --steps 3 --warmup 1
echo done
