#!/bin/bash
# Frame timelines (rocprofv3 kernel trace, last uninstrumented C3 frame) of
# env-selected variants.  VARIANTS="name:ENV=val+ENV2=val ..."; BENCH_EXTRA
# adds bench.py arguments.  Outputs gpurun_out/tl_<name>.txt.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-default:X=1}; do
  name=${v%%:*}; envs=${v#*:}; envs=${envs//+/ }
  env $envs timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu ${BENCH_EXTRA:-} > gpurun_out/tlb_$name.log 2>&1
  rc=$?; echo "bench $name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/tlb_$name.log; exit $rc; fi
  python -c "import json; d=json.loads(open('gpurun_out/tlb_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], 'Mrays/s', d['ms_per_step'], 'ms')"
  # rocprofv3 must exec python directly (no env hop): export the variant's variables
  ( export $envs; timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tlp_$name -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-times ${BENCH_EXTRA:-} > gpurun_out/tlp_$name.log 2>&1 )
  rc=$?; echo "prof $name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/tlp_$name.log; exit $rc; fi
  python3 tools/frame_timeline.py gpurun_out/tlp_$name > gpurun_out/tl_$name.txt 2>&1
  rm -rf gpurun_out/tlp_$name
done
