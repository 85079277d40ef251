#!/bin/bash
# Driver settings (K = 20, W = 5): one frame at a time vs four in flight, at N = 1 and at the
# per-rank shares of N = 2 / 4 / 8 (--shard-of).
set -u
O=gpurun_out/s5; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['avg_kernel_ms'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --steps 20 --warmup 5"
for i in 1 2 3; do
  run n1_f1_$i $B --inflight 1
  run n1_f4_$i $B --inflight 4
done
for s in 2 4 8; do
  run sh${s}_f1 $B --inflight 1 --shard-of $s
  run sh${s}_f4 $B --inflight 4 --shard-of $s
done
#!/bin/bash
# C4 where the time goes: single-stream frame timeline (tuning split=0) and the default
# two-stream one, rocprofv3 kernel trace, one frame at a time.
set -u
O=gpurun_out/s6; mkdir -p $O
for v in "single:split=0" "default:"; do
  name=${v%%:*}; tune=${v#*:}
  ( export RT_TUNE=$tune; timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p_$name -o run --output-format csv -- \
      python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu --no-kernel-times --no-gather > $O/p_$name.log 2>&1 ) || { echo "prof $name failed"; tail -5 $O/p_$name.log; exit 1; }
  python3 tools/frame_timeline.py $O/p_$name > $O/tl_c4_$name.txt 2>&1
  rm -rf $O/p_$name
  echo "$name done"; tail -1 $O/p_$name.log | cut -c1-160
done
