set -u
mkdir -p gpurun_out/lds
export TMPDIR=/tmp
(rocprofv3 -L 2>&1 || true) | grep -i "lds\|SQ_INST_LEVEL\|SQC_LDS" > gpurun_out/lds/counters.txt 2>&1 || true
RT_TUNE=split=0 RT_LIBRTAMD=/root/repo/rust-raytrace_amd/librtamd_st.so timeout -k 10 300 python tools/stamp_probe.py --tune split=0 > gpurun_out/lds/stamp_single.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/lds/p1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-times --no-gather > gpurun_out/lds/p1.log 2>&1
echo pmc rc=$?
cat gpurun_out/lds/stamp_single.txt
