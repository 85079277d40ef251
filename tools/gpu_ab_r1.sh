#!/bin/bash
# Same-box A/B of the current build against an older tree in old_r1/
# (gitignored; e.g. `git worktree add /tmp/r1 <commit>`, build it there, copy it
# without .git to old_r1/): C4 and C3, alternating, plus tuning variants.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/abr1
mkdir -p $O
run() { local name=$1 dir=$2; shift 2; ( cd $dir && timeout -k 10 300 python bench.py --no-cpu --steps 8 --warmup 2 "$@" ) > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(tail -1 $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms", d["value"], {k: v["ms_per_frame"] for k, v in (d["roofline"]["kernels"] or {}).items()})')"; [ $rc -eq 0 ] || exit $rc; }
for cfg in ${CFGS:-c4 c3}; do
  [ "${NO_NOGRID:-0}" = 1 ] && true
  run ${cfg}_new . --config $cfg --no-gather
  run ${cfg}_old old_r1 --config $cfg
  run ${cfg}_new2 . --config $cfg --no-gather
  run ${cfg}_old2 old_r1 --config $cfg
  RT_TUNE=grid_occ=0 run ${cfg}_nogrid . --config $cfg --no-gather
done
echo done
