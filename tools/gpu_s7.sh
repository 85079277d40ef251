#!/bin/bash
# C4 schedule A/B with binary16 nodes: one stream vs the two B streams, CU-masked B streams, one B stream.
set -u
O=gpurun_out/s7; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --config c4 --steps 4 --warmup 1"
for i in 1 2; do
  run def_$i $B
  run split0_$i RT_TUNE=split=0 $B
done
run cu2 RT_TUNE=cu_mask=2 $B
run cu3 RT_TUNE=cu_mask=3 $B
run cu4 RT_TUNE=cu_mask=4 $B
run b1 RT_TUNE=bstreams=1 $B
run prio1 RT_TUNE=prio=1 $B
B5="python bench.py --no-cpu --no-kernel-times --no-gather --config c5 --steps 2 --warmup 1"
run c5_def $B5
run c5_split0 RT_TUNE=split=0 $B5
