#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, --kernel-trace only,
# as MI355X_MICROARCH.md / gpurun require).  Usage: tools/gpu_pmc.sh [bench args]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
ARGS="${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmc/p$i -o run --output-format csv -- \
      python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
