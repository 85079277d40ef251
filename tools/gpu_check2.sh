#!/bin/bash
# Round-2 check: GPU parity suite, smoke, default bench, a 2-rank launcher
# rehearsal (gloo, both ranks on the one card).  Each GPU step has its own limit.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/check2
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 600 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -c 400 $O/$name.log | tail -2; [ $rc -eq 0 ] || exit $rc; }
python -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null
step pytest python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
step smoke python -c "import __graft_entry__ as g; g.smoke()"
step bench python bench.py
step bench2 python bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 3
echo done
