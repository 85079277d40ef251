#!/bin/bash
# One GPU session = a list of steps run in order.  Every GPU step has its own
# time limit; a failing step ends the session (no retries: a fault, abort or
# time limit means read the logs, fix, run again).  Outputs: gpurun_out/$S/
# (S defaults to "s").  Replaces round 1-2's one-off gpu_s*.sh scripts.
#
#   test:<pytest -k expression | all>          pytest -m gpu (thread timeouts, one process)
#   smoke                                      __graft_entry__.smoke()
#   bench:<name>:[ENV=v ...] <bench.py args>   one bench line -> <name>.log, prints ms and value
#   prof:<name>:[ENV=v ...] <bench.py args>    rocprofv3 --kernel-trace --stats -> <name>/, kernel_stats
#                                              summary <name>.stats.txt and the last frame's timeline
#                                              <name>.timeline.txt
#   run:<name>:[ENV=v ...] <command>          any other GPU command (e.g. python3 tools/stamp_probe.py) -> <name>.log
#   pmcx:<name>:<counters>:<program args>      ONE --pmc pass over another program (the binary itself after --)
#   pmc:<name>:<counters, space separated>:<bench.py args>   ONE --pmc pass (--kernel-trace only)
#                                              -> <name>/ and a per-kernel summary <name>.txt
#
#   e.g. S=c4prof tools/gpu.sh 'test:fullsize' 'bench:c4:--config c4 --steps 4 --warmup 1 --no-cpu' \
#        'pmc:c4_sq1:SQ_WAVES SQ_INSTS_VALU:--config c4 --steps 1 --warmup 1 --no-cpu --no-kernel-times'
#
# A variant library built with `make BUILD=build_x LIB=librtamd_x.so EXTRA=-D...` is selected per step
# with RT_LIBRTAMD=rust-raytrace_amd/librtamd_x.so; schedule knobs with RT_TUNE=key=v,key=v.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${S:-s}
mkdir -p "$O"
export TMPDIR=/tmp
QUIET="--no-gather"

line() {  # ms_per_step and value of a bench log's JSON line
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['ms_per_step'], 'ms', d['value'], d['unit'])" "$1"
}

split_env() {  # "A=1 B=2 --x y" -> ENVS="A=1 B=2", REST="--x y"
  ENVS=""; REST=""
  local w
  for w in $1; do
    if [ -z "$REST" ] && [[ "$w" == [A-Z]*=* ]]; then ENVS="$ENVS $w"; else REST="$REST $w"; fi
  done
}

for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  case "$kind" in
  test)
    expr=$rest
    if [ "$expr" = "all" ]; then k=(); else k=(-k "$expr"); fi
    timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread "${k[@]}" \
        > "$O/pytest.log" 2>&1
    rc=$?; echo "test [$expr] rc=$rc: $(tail -1 "$O/pytest.log")"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$O/pytest.log" | head -20; exit $rc; }
    ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc: $(tail -1 "$O/smoke.log")"; [ $rc -eq 0 ] || exit $rc
    ;;
  bench)
    name=${rest%%:*}; split_env "${rest#*:}"
    env $ENVS timeout -k 10 600 python bench.py $QUIET $REST > "$O/$name.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "bench $name rc=$rc"; tail -5 "$O/$name.log"; exit $rc; }
    echo "bench $name [$ENVS ]: $(line "$O/$name.log")"
    ;;
  prof)
    name=${rest%%:*}; split_env "${rest#*:}"
    # rocprofv3 must start python itself (no env hop): export the step's variables in a subshell
    ( [ -n "$ENVS" ] && export $ENVS
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- \
          python3 bench.py $QUIET --no-cpu --no-kernel-times $REST > "$O/$name.log" 2>&1 )
    rc=$?
    [ $rc -eq 0 ] || { echo "prof $name rc=$rc"; tail -5 "$O/$name.log"; exit $rc; }
    python3 tools/prof_summary.py "$O/$name" > "$O/$name.stats.txt" 2>&1
    python3 tools/frame_timeline.py "$O/$name" > "$O/$name.timeline.txt" 2>&1
    echo "prof $name [$ENVS ]: $(line "$O/$name.log"); $(head -1 "$O/$name.stats.txt" | cut -c1-150)"
    ;;
  pmc)
    name=${rest%%:*}; r2=${rest#*:}; ctrs=${r2%%:*}; args=${r2#*:}
    timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-trace -d "$O/$name/p1" -o run --output-format csv -- \
        python3 bench.py $QUIET --no-cpu --no-kernel-times $args > "$O/$name.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "pmc $name rc=$rc"; tail -5 "$O/$name.log"; exit $rc; }
    python3 tools/pmc_summary.py "$O/$name" > "$O/$name.txt" 2>&1
    echo "pmc $name ($ctrs) ok"
    ;;
  pmcx)
    name=${rest%%:*}; r2=${rest#*:}; ctrs=${r2%%:*}; cmd=${r2#*:}
    timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-trace -d "$O/$name/p1" -o run --output-format csv -- \
        $cmd > "$O/$name.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "pmcx $name rc=$rc"; tail -5 "$O/$name.log"; exit $rc; }
    python3 tools/pmc_summary.py "$O/$name" > "$O/$name.txt" 2>&1
    echo "pmcx $name ($ctrs) ok"
    ;;
  run)
    name=${rest%%:*}; split_env "${rest#*:}"
    env $ENVS timeout -k 10 600 $REST > "$O/$name.log" 2>&1
    rc=$?; echo "run $name rc=$rc: $(tail -1 "$O/$name.log" | cut -c1-200)"; [ $rc -eq 0 ] || { tail -5 "$O/$name.log"; exit $rc; }
    ;;
  *)
    echo "unknown step kind: $kind"; exit 2
    ;;
  esac
done
echo "session done"
