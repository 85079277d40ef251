#!/bin/bash
# HBM traffic per render at C4 and C5 (FETCH_SIZE / WRITE_SIZE, separate passes).
set -u
export TMPDIR=/tmp
PMC_OUT=gpurun_out/s17/pmc_c4 GROUPS_PMC="FETCH_SIZE;WRITE_SIZE" BENCH_ARGS="--config c4 --steps 1 --warmup 1 --no-cpu --no-kernel-times --no-gather" bash tools/gpu_pmc.sh || exit $?
PMC_OUT=gpurun_out/s17/pmc_c5 GROUPS_PMC="FETCH_SIZE;WRITE_SIZE" BENCH_ARGS="--config c5 --steps 1 --warmup 1 --no-cpu --no-kernel-times --no-gather" bash tools/gpu_pmc.sh || exit $?
for d in gpurun_out/s17/pmc_c4 gpurun_out/s17/pmc_c5; do rm -f $d/p*/run_kernel_trace.csv; done
