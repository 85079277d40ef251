#!/bin/bash
# End-of-milestone GPU session: parity suite, smoke, headline bench, rocprofv3
# kernel stats + frame timeline, PMC passes (HBM traffic, SQ counters), and the
# C1 path-kernel bench + kernel stats.  Every GPU step has its own time limit;
# a fatal exit (fault, abort, timeout) ends the script.  Outputs: gpurun_out/round/.
# Profiling passes render one frame at a time (--inflight 1): their per-frame
# split of the kernel trace assumes frames do not interleave.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/round
mkdir -p $O
export TMPDIR=/tmp
fatal() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -gt 1 ]; then echo "fatal: $what"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
fatal $? pytest; tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fatal $? smoke; tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
fatal $? bench; tail -1 $O/bench.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu --no-kernel-times --inflight 1 > $O/prof.log 2>&1
fatal $? rocprof
python3 tools/prof_summary.py $O/prof > $O/kernel_stats.txt 2>&1
python3 tools/frame_timeline.py $O/prof > $O/frame_timeline.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu --inflight 1 > $O/bench_f1.log 2>&1
fatal $? bench_f1; tail -1 $O/bench_f1.log | cut -c1-200
PMC_OUT=$O/pmc GROUPS_PMC="FETCH_SIZE;WRITE_SIZE" BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-kernel-times --inflight 1" bash tools/gpu_pmc.sh
fatal $? pmc_traffic
PMC_OUT=$O/pmc_sq GROUPS_PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-kernel-times --inflight 1" bash tools/gpu_pmc.sh
fatal $? pmc_sq
python3 tools/pmc_summary.py $O/pmc_sq > $O/pmc_sq.txt 2>&1
timeout -k 10 300 python bench.py --config c1 > $O/bench_c1.log 2>&1
fatal $? bench_c1; tail -1 $O/bench_c1.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o run --output-format csv -- \
    python3 bench.py --config c1 --no-cpu > $O/prof_c1.log 2>&1
fatal $? rocprof_c1
timeout -k 10 400 python bench.py --config c4 > $O/bench_c4.log 2>&1
fatal $? bench_c4; tail -1 $O/bench_c4.log | cut -c1-200
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.log 2>&1
fatal $? bench_c5; tail -1 $O/bench_c5.log | cut -c1-200
VARIANTS="single:RT_TUNE=split=0" BENCH_EXTRA="--inflight 1" bash tools/gpu_timeline.sh > $O/tl.log 2>&1
fatal $? timeline_single; cp gpurun_out/tl_single.txt $O/frame_timeline_single.txt
echo done
