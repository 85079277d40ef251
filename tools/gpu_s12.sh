#!/bin/bash
set -u
O=gpurun_out/s12; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/schedule_probe.py > $O/probe.log 2>&1 || exit $?; cat $O/probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "deep_tree or half_node" > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -1 $O/pytest.log
