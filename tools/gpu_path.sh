set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --config c1 > gpurun_out/bench_c1.log 2>&1 || { echo bench_c1 fail; tail -20 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run --output-format csv -- python3 bench.py --config c1 --no-cpu > gpurun_out/prof_c1.log 2>&1 || { echo prof fail; exit 1; }
find gpurun_out/prof_c1 -name "*kernel_stats*"
