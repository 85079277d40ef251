#!/bin/bash
# GPU tests + A/B bench of env-selected variants.  VARIANTS="name:ENV=val ..."
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
fi
for v in ${VARIANTS:-default:X=1}; do
  name=${v%%:*}; envs=${v#*:}; envs=${envs//+/ }
  if [ "${VTESTS:-0}" = "1" ]; then
    env $envs timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -m gpu \
        -k "config3 or axis_aligned or extreme or ten_thousand or bit_for_bit or golden" > gpurun_out/vtest_$name.log 2>&1
    rc=$?; echo "vtests $name rc=$rc: $(tail -1 gpurun_out/vtest_$name.log)"; if [ $rc -gt 1 ]; then exit $rc; fi
  fi
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu ${BENCH_EXTRA:-} > gpurun_out/bench_$name.log 2>&1
  rc=$?; echo "bench $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_$name.log; exit $rc; fi
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], 'Mrays/s', d['ms_per_step'], 'ms')"
  if [ "${PROF:-0}" = "1" ]; then
    env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_$name.log 2>&1
    rc=$?; echo "prof $name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  fi
done
