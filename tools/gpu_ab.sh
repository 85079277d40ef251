#!/bin/bash
# GPU tests + A/B bench of env-selected variants.  VARIANTS="name:ENV=val ..."
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for v in ${VARIANTS:-default:X=1}; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_$name.log 2>&1
  rc=$?; echo "bench $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_$name.log; exit $rc; fi
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], 'Mrays/s', d['ms_per_step'], 'ms')"
done
