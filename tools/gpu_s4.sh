#!/bin/bash
# Half-node prefix source (src 5) vs f32 nodes (src 8) at C4 / C5; parity first.
set -u
O=gpurun_out/s4; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "half_node or ten_thousand or config5 or tuning or multi_chunk" > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather"
for i in 1 2; do
  run c4_half_$i $B --config c4 --steps 5 --warmup 2
  run c4_f32_$i RT_TUNE=half_nodes=0 $B --config c4 --steps 5 --warmup 2
done
run c4_half_pfx32 RT_TUNE=prefix_kb=32 $B --config c4 --steps 5 --warmup 2
run c4_half_pfx96 RT_TUNE=prefix_kb=96 $B --config c4 --steps 5 --warmup 2
run c5_half $B --config c5 --steps 3 --warmup 1
run c5_f32 RT_TUNE=half_nodes=0 $B --config c5 --steps 3 --warmup 1
