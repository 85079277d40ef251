#!/bin/bash
# End-of-round check, then A/B: nearest-hit waves at s_setprio 3 (librtamd_r5) vs 2 at C3 and C4.
set -u
bash tools/gpu_final.sh || exit $?
O=gpurun_out/s19; mkdir -p $O; export TMPDIR=/tmp
L=rust-raytrace_amd
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --steps 20 --warmup 5"
for i in 1 2 3; do
  run c3_p2_$i $B
  run c3_p3_$i RT_LIBRTAMD=$L/librtamd_r5.so $B
done
run c4_p2 $B --config c4 --steps 4 --warmup 1
run c4_p3 RT_LIBRTAMD=$L/librtamd_r5.so $B --config c4 --steps 4 --warmup 1
