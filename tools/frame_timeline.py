"""Per-launch timeline of the last uninstrumented wavefront frame of a
rocprofv3 --kernel-trace run (directory argument)."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
tr.sort(key=lambda t: int(t["Start_Timestamp"]))
starts = [i for i, t in enumerate(tr) if "wf_nearest" in t["Kernel_Name"] and ", true, false>" in t["Kernel_Name"]]
i0 = starts[-1]
t0 = int(tr[i0]["Start_Timestamp"])
for t in tr[i0:]:
    s = (int(t["Start_Timestamp"]) - t0) / 1e3
    dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3
    name = t["Kernel_Name"].replace("rtamd::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    print(f"{s:8.1f} {dur:8.1f}  {name}")
    if "wf_tally" in name:
        break
