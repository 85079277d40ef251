#!/bin/bash
# C4 where the time goes: single-stream frame timeline (tuning split=0) and the default
# two-stream one, rocprofv3 kernel trace, one frame at a time.
set -u
O=gpurun_out/s6; mkdir -p $O; export TMPDIR=/tmp
for v in "single:split=0" "default:"; do
  name=${v%%:*}; tune=${v#*:}
  ( export RT_TUNE=$tune; timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p_$name -o run --output-format csv -- \
      python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu --no-kernel-times --no-gather > $O/p_$name.log 2>&1 ) || { echo "prof $name failed"; tail -5 $O/p_$name.log; exit 1; }
  python3 tools/frame_timeline.py $O/p_$name > $O/tl_c4_$name.txt 2>&1
  rm -rf $O/p_$name
  echo "$name done"; tail -1 $O/p_$name.log | cut -c1-160
done
