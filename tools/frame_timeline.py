"""Per-launch timeline of the last timed-loop wavefront frame of a rocprofv3
--kernel-trace run of bench.py (directory argument): the last uninstrumented
frame before the RT_COUNT_WORK render (the PCIe-inclusive rt_render calls come
after it); start (us from the frame's first launch), duration (us), stream,
kernel; up to the frame-end fold."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
tr.sort(key=lambda t: int(t["Start_Timestamp"]))


def targs(name):
    return [a.strip() for a in name.split("<", 1)[1].split(">")[0].split(",")] if "<" in name else []


# generation 0 of an uninstrumented frame: wf_nearest<src, kCam = true, kCount = false, ...>
gen0 = [i for i, t in enumerate(tr) if "wf_nearest<" in t["Kernel_Name"] and targs(t["Kernel_Name"])[1:2] == ["true"]]
inst = next((i for i in gen0 if targs(tr[i]["Kernel_Name"])[2] == "true"), len(tr))
starts = [i for i in gen0 if i < inst]
i0 = starts[-1]
t0 = int(tr[i0]["Start_Timestamp"])
for j, t in enumerate(tr[i0:]):
    if j > 0 and "wf_nearest<" in t["Kernel_Name"] and targs(t["Kernel_Name"])[1:2] == ["true"]:
        break                                      # the next frame (e.g. the instrumented one)
    s = (int(t["Start_Timestamp"]) - t0) / 1e3
    dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3
    name = t["Kernel_Name"].replace("rtamd::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    q = t.get("Stream_Id") or t.get("Queue_Id") or ""
    print(f"{s:8.1f} {dur:8.1f}  {q:>3}  {name}")
    if name.startswith("wf_fold<"):               # the frame-end fold (after the tally since round 3)
        break
