#!/bin/bash
# Per-rank time of an N-rank frame on one GPU (--shard-of N: rank 0's row bands), C3 and C4, and
# the two-rank launcher rehearsal (gloo, both ranks on the one card).
set -u
O=gpurun_out/s9; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['n_gpus'], d['config']['ranks'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather"
run c3_n1 $B --steps 20 --warmup 5
for s in 2 4 8; do run c3_sh$s $B --steps 20 --warmup 5 --shard-of $s; done
run c4_n1 $B --config c4 --steps 4 --warmup 1
for s in 2 4 8; do run c4_sh$s $B --config c4 --steps 4 --warmup 1 --shard-of $s; done
run gloo2 python bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 5 --warmup 2
