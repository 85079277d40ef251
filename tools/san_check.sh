#!/bin/bash
# Host-code sanitizer run (ASan + UBSan, gcc runtime): builds librtamd_san.so
# (make SAN=1) and runs the CPU tests that drive the host C++ through the C ABI
# -- the scene parser (serialize.rs replacement), the texture decoder, the BVH
# and light-grid builders, the BMP writer -- with the sanitizer runtime preloaded.
# No GPU: device entry points fail with RT_E_NODEVICE, as in the plain CPU suite.
set -eu
cd "$(dirname "$0")/.."
make -s -C rust-raytrace_amd SAN=1 BUILD=/tmp/rtamd_san LIB=/tmp/rtamd_san/librtamd_san.so -j8
ASAN_SO=$(gcc -print-file-name=libasan.so)
UBSAN_SO=$(gcc -print-file-name=libubsan.so)
export RT_LIBRTAMD=/tmp/rtamd_san/librtamd_san.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$ASAN_SO $UBSAN_SO" python -m pytest -q -p no:cacheprovider \
    tests/test_host.py tests/test_lightgrid.py tests/test_oracle.py tests/test_fixtures.py "$@"
