"""One timed-loop frame's host API calls beside its kernels:
from a rocprofv3 --kernel-trace --hip-runtime-trace run of bench.py, every
hipLaunchKernel of the frame with its host start and duration and its kernel's
device start (both from the frame's first kernel start) and queue, and the
other HIP calls between them.  Shows whether the host keeps ahead of the
device (launches enqueued long before their kernels start) and what the
frame boundary holds.

    python3 tools/api_timeline.py gpurun_out/<dir>
"""
import csv
import sys


def main():
    d = sys.argv[1]
    api = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
    kt = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    byc = {k["Correlation_Id"]: k for k in kt}
    kt.sort(key=lambda t: int(t["Start_Timestamp"]))
    g0 = [t for t in kt if "wf_nearest<22, true, false" in t["Kernel_Name"] or "wf_nearest<23, true, false" in t["Kernel_Name"]]
    a, b = int(g0[-3]["Start_Timestamp"]), int(g0[-2]["Start_Timestamp"])
    print(f"frame: generation 0 at device t = 0, the next frame's at {(b - a) / 1e3:.1f} us")
    print(f"{'host us':>9} {'call us':>8} {'kernel us':>10} queue  call / kernel")
    calls = sorted((x for x in api if a - 800000 <= int(x["Start_Timestamp"]) <= b), key=lambda x: int(x["Start_Timestamp"]))
    for x in calls:
        if x["Function"] == "hipGetLastError":
            continue
        k = byc.get(x["Correlation_Id"]) if x["Function"] == "hipLaunchKernel" else None
        name = k["Kernel_Name"].replace("rtamd::(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:44] if k else ""
        ks = f"{(int(k['Start_Timestamp']) - a) / 1e3:10.1f}" if k else " " * 10
        q = k.get("Queue_Id", "") if k else ""
        print(f"{(int(x['Start_Timestamp']) - a) / 1e3:9.1f} {(int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3:8.1f} "
              f"{ks} {q:>5}  {x['Function']} {name}")


if __name__ == "__main__":
    main()
