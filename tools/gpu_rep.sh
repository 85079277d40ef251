#!/bin/bash
# Repeated A/B benches in one box session: VARIANTS="name:ENV=val+ENV=val|bench args ..." (spaces in args as ,)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for v in ${VARIANTS}; do
  name=${v%%:*}; rest=${v#*:}; envs=${rest%%|*}; args=""
  if [[ "$rest" == *"|"* ]]; then args=${rest#*|}; args=${args//,/ }; fi
  envs=${envs//+/ }
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu $args > gpurun_out/rep_$name.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 gpurun_out/rep_$name.log; exit $rc; fi
  python -c "import json; d=json.loads(open('gpurun_out/rep_$name.log').read().strip().splitlines()[-1]); print('rep $rep', '$name', round(d['value']), 'Mrays/s', d['ms_per_step'], 'ms')"
done
done
