#!/bin/bash
# Frames in flight x hardware queues at N = 1 (C3) and at a 1/8 shard (per-rank work of N = 8).
set -u
O=gpurun_out/s3; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --steps 24 --warmup 6"
for q in 4 8 16 24; do for f in 1 2 3 4 6; do
  run n1_q${q}_f$f GPU_MAX_HW_QUEUES=$q $B --inflight $f
  run sh8_q${q}_f$f GPU_MAX_HW_QUEUES=$q $B --inflight $f --shard-of 8
done; done
