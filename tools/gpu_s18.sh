#!/bin/bash
# A/B: wide-code compact stack entries (src 3, librtamd_r4) vs src 5 at C5; schedule probe and
# the C5-class parity tests on the r4 build first.
set -u
O=gpurun_out/s18; mkdir -p $O; export TMPDIR=/tmp
L=rust-raytrace_amd
RT_LIBRTAMD=$L/librtamd_r4.so timeout -k 10 200 python - > $O/probe.log 2>&1 <<'PY' || { cat $O/probe.log; exit 1; }
import sys
sys.path[:0] = [".", "rust-raytrace_amd"]
import libraytrace as lr
from libraytrace import scenes
for name, spec in (("c5", scenes.config5(64, 64)), ("c4", scenes.config4(64, 64))):
    with lr.Context(0) as ctx:
        ctx.set_tuning("verbose", 1)
        ctx.upload(lr.Scene.deserialize(spec.to_text()))
        print(name, flush=True)
        ctx.render(lr.render_opts(spec.width, spec.height, max_depth=spec.max_depth, spp=1, algo=lr.RT_ALGO_WAVEFRONT))
        sys.stderr.flush()
PY
cat $O/probe.log
RT_LIBRTAMD=$L/librtamd_r4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "half_node or ten_thousand or config5 or chain or tuning" > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"; }
B="python bench.py --no-cpu --no-kernel-times --no-gather --config c5 --steps 2 --warmup 1"
for i in 1 2; do
  run c5_src5_$i $B
  run c5_src3_$i RT_LIBRTAMD=$L/librtamd_r4.so $B
done
