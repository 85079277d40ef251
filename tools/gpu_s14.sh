#!/bin/bash
# rocprofv3 kernel stats of the C4 and C5 benches on the final build (one stream, binary16 prefix source).
set -u
O=gpurun_out/s14; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- \
    python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-gather > $O/prof_c4.log 2>&1 || { tail -5 $O/prof_c4.log; exit 1; }
python3 tools/prof_summary.py $O/prof_c4 > $O/c4_kernel_stats.txt 2>&1; head -12 $O/c4_kernel_stats.txt; tail -1 $O/prof_c4.log | cut -c1-200
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- \
    python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu --no-gather --no-kernel-times > $O/prof_c5.log 2>&1 || { tail -5 $O/prof_c5.log; exit 1; }
python3 tools/prof_summary.py $O/prof_c5 > $O/c5_kernel_stats.txt 2>&1; head -12 $O/c5_kernel_stats.txt
rm -f $O/prof_c4/run_kernel_trace.csv $O/prof_c5/run_kernel_trace.csv
