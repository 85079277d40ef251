#!/bin/bash
# C5 chunking: the default 80 GB working-set cap (7 chunks of ~38 M px) vs 4 and 3 chunks.
set -u
O=gpurun_out/s10; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --config c5 --steps 3 --warmup 1"
run c5_def $B
run c5_4ch RT_TUNE=chunk_pixels=67108864 $B
run c5_3ch RT_TUNE=chunk_pixels=89478486 $B
run c5_def2 $B
