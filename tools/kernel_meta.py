"""Register / scratch / LDS usage of the gfx950 kernels in a hipcc object or
shared library (its .hip_fatbin offload bundle), from the code object's
metadata notes.  Usage: python3 tools/kernel_meta.py build/trace_kernel.o [name-substring]"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
obj, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
with tempfile.TemporaryDirectory() as d:
    fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
    subprocess.run([B + "/llvm-objcopy", "--dump-section", ".hip_fatbin=" + fb, obj, os.path.join(d, "junk")], check=True)
    subprocess.run([B + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fb,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
    notes = subprocess.run([B + "/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
cur = {}
rows = []
for line in notes.splitlines():
    s = line.strip()
    m = re.match(r"^-?\s*\.(\w+):\s*(.*)$", s)
    if not m:
        continue
    k, v = m.group(1), m.group(2).strip("'")
    if k == "args":
        if cur:
            rows.append(cur)
        cur = {}
    cur[k] = v
if cur:
    rows.append(cur)
for r in rows:
    name = r.get("name", "")
    if pat and pat not in name:
        continue
    if ".kd" in name or not name:
        continue
    print(f"{name[:90]:90s} vgpr {r.get('vgpr_count','?'):>4} agpr {r.get('agpr_count','?'):>3} sgpr {r.get('sgpr_count','?'):>4} "
          f"vspill {r.get('vgpr_spill_count','?'):>3} sspill {r.get('sgpr_spill_count','?'):>3} "
          f"scratch {r.get('private_segment_fixed_size','?'):>4} lds {r.get('group_segment_fixed_size','?')}")
