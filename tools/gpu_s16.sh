#!/bin/bash
# Final build with src 6: full GPU suite, smoke, driver bench line, C4 and C5 benches.
set -u
O=gpurun_out/s16; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?; tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?; tail -1 $O/bench.log | cut -c1-200
timeout -k 10 400 python bench.py --config c4 > $O/bench_c4.log 2>&1 || exit $?; tail -1 $O/bench_c4.log | cut -c1-200
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.log 2>&1 || exit $?; tail -1 $O/bench_c5.log | cut -c1-200
timeout -k 10 300 python bench.py --config c4 --shard-of 8 --no-cpu --no-gather --steps 4 --warmup 1 > $O/c4_sh8.log 2>&1 || exit $?; tail -1 $O/c4_sh8.log | cut -c1-200
