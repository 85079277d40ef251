#!/bin/bash
# Camera view of trees beyond LDS: top 64 KB staged in LDS (default) vs all from L2 (cam_prefix_kb=0).
set -u
O=gpurun_out/s20; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "half_node or ten_thousand or config5 or chain or tuning or multi_chunk" > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --config c4 --steps 4 --warmup 1"
for i in 1 2 3; do
  run c4_pfx64_$i $B
  run c4_pfx0_$i RT_TUNE=cam_prefix_kb=0 $B
done
run c4_pfx32 RT_TUNE=cam_prefix_kb=32 $B
B5="python bench.py --no-cpu --no-kernel-times --no-gather --config c5 --steps 2 --warmup 1"
run c5_pfx64 $B5
run c5_pfx0 RT_TUNE=cam_prefix_kb=0 $B5
