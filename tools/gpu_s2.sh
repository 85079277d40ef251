#!/bin/bash
# A/B session: compact nearest-hit stack (src 9) vs 64-bit entries (src 7) at C3, and
# frames in flight with more hardware queues at a 1/8 shard.  Each GPU step has its own limit.
set -u
O=gpurun_out/s2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "tuning or config3 or golden or fixtures or ten_thousand" > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --steps 20 --warmup 5"
for i in 1 2 3; do
  run c3_compact_$i $B
  run c3_wide_$i RT_TUNE=compact_stack=0 $B
done
run sh8_q16_f1 GPU_MAX_HW_QUEUES=16 $B --shard-of 8
run sh8_q16_f2 GPU_MAX_HW_QUEUES=16 $B --shard-of 8 --inflight 2
run sh8_q16_f4 GPU_MAX_HW_QUEUES=16 $B --shard-of 8 --inflight 4
run sh8_q16_f4_b1 GPU_MAX_HW_QUEUES=16 RT_TUNE=bstreams=1 $B --shard-of 8 --inflight 4
run sh8_q4_f1 $B --shard-of 8
run sh8_q4_f1_wide RT_TUNE=compact_stack=0 $B --shard-of 8
