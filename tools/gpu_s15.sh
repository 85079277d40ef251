#!/bin/bash
# A/B: 18-bit compact stack entries for the binary16 prefix source (src 6, librtamd_r3) vs src 5, at C4;
# parity of the C4-class tests on the r3 build first.
set -u
O=gpurun_out/s15; mkdir -p $O; export TMPDIR=/tmp
L=rust-raytrace_amd
RT_LIBRTAMD=$L/librtamd_r3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "half_node or ten_thousand or tuning or chain or config5" > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --config c4 --steps 4 --warmup 1"
for i in 1 2 3; do
  run c4_src5_$i $B
  run c4_src6_$i RT_LIBRTAMD=$L/librtamd_r3.so $B
done
