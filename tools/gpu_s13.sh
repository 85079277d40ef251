#!/bin/bash
# A/B: register entries on top of the compact stack (librtamd_r1 / _r2 builds) vs the default (0).
set -u
O=gpurun_out/s13; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --steps 20 --warmup 5"
L=rust-raytrace_amd
for i in 1 2 3; do
  run r0_$i $B
  run r1_$i RT_LIBRTAMD=$L/librtamd_r1.so $B
  run r2_$i RT_LIBRTAMD=$L/librtamd_r2.so $B
done
