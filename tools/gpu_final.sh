#!/bin/bash
# End-of-round check on the committed tree: GPU suite, smoke, the driver's bench line, gloo launcher rehearsal.
set -u
O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?; tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?; tail -1 $O/bench.log | cut -c1-240
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 > $O/bench_gloo2.log 2>&1 || exit $?; tail -1 $O/bench_gloo2.log | cut -c1-240
