set -u
O=gpurun_out/s1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?; tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?; tail -1 $O/bench.log | cut -c1-400
for v in "--shard-of 8" "--shard-of 8 --inflight 2" "--shard-of 8 --inflight 4" "--shard-of 4 --inflight 2" "--inflight 2"; do
  timeout -k 10 200 python bench.py --no-cpu --no-kernel-times --no-gather --steps 20 --warmup 5 $v > $O/sh.log 2>&1 || exit $?
  echo "$v: $(python -c "import json,sys; d=json.loads(open('$O/sh.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
done
