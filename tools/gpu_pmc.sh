#!/bin/bash
# PMC passes: each counter group in its own rocprofv3 run with --kernel-trace
# only (no sys/runtime traces), as MI355X_MICROARCH.md and gpurun require.
# GROUPS (';'-separated counter lists) and BENCH_ARGS may be overridden.
set -u
cd "$(dirname "$0")/.."
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu}"
DEFAULT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum"
IFS=';' read -ra GRPS <<< "${GROUPS_PMC:-$DEFAULT}"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
      python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
