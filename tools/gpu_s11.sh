#!/bin/bash
# Full GPU suite + smoke on the final build; which stack / source / stream schedule the host picks
# for the deep-chain test scene, C3 and C4 (tuning verbose=1).
set -u
O=gpurun_out/s11; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?; tail -1 $O/smoke.log
timeout -k 10 300 python tools/schedule_probe.py > $O/probe.log 2>&1 || exit $?; cat $O/probe.log
