#!/bin/bash
# Compact per-kernel resource usage (VGPRs, scratch bytes/lane, SGPR/VGPR spills,
# waves/SIMD) of trace_kernel.hip for gfx950; optional grep filter on the name.
cd "$(dirname "$0")/../rust-raytrace_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -I../include -Icsrc \
  $EXTRA -c csrc/trace_kernel.hip -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/ \[-Rpass.*//' |
  awk '/Function Name:/{n=$NF} / VGPRs:/{v=$NF} /ScratchSize/{s=$NF} /SGPRs Spill/{ss=$NF} /VGPRs Spill/{vs=$NF}
       /Occupancy/{print n, "vgpr=" v, "scratch=" s, "sspill=" ss, "vspill=" vs, "occ=" $NF}' |
  sed 's/_ZN5rtamd12_GLOBAL__N_1//; s/EEEvNS_8DevScene[^ ]*//' | grep -E "${1:-.}"
