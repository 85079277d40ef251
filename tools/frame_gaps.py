"""Where one timed-loop frame's time goes between kernels: from a
rocprofv3 --kernel-trace run of bench.py, the last uninstrumented frame's kernels
(start and duration in us from the frame's first launch, queue), the gap before
it (the previous frame's last kernel end -> its first kernel start), its span
(first start -> last end), and on each queue the busy time and the idle gaps
between its kernels.

    python3 tools/frame_gaps.py gpurun_out/<prof dir>
"""
import csv
import sys


def targs(name):
    return [a.strip() for a in name.split("<", 1)[1].split(">")[0].split(",")] if "<" in name else []


def is_gen0(t):
    return "wf_nearest<" in t["Kernel_Name"] and targs(t["Kernel_Name"])[1:2] == ["true"]


def main():
    d = sys.argv[1]
    tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    tr.sort(key=lambda t: int(t["Start_Timestamp"]))
    gen0 = [i for i, t in enumerate(tr) if is_gen0(t)]
    inst = next((i for i in gen0 if targs(tr[i]["Kernel_Name"])[2] == "true"), len(tr))
    starts = [i for i in gen0 if i < inst]
    i0 = starts[-1]
    i1 = next((i for i in gen0 if i > i0), len(tr))
    frame = [t for t in tr[i0:i1] if "wf_" in t["Kernel_Name"] or "rows_to_host" in t["Kernel_Name"]]
    t0 = int(tr[i0]["Start_Timestamp"])
    prev_end = max((int(t["End_Timestamp"]) for t in tr[:i0]), default=t0)
    q = lambda t: t.get("Stream_Id") or t.get("Queue_Id") or ""
    span_end = max(int(t["End_Timestamp"]) for t in frame)
    print(f"gap before the frame (previous kernel end -> first start): {(t0 - prev_end) / 1e3:.1f} us")
    print(f"frame span (first start -> last end): {(span_end - t0) / 1e3:.1f} us, {len(frame)} kernels")
    byq = {}
    for t in frame:
        s = (int(t["Start_Timestamp"]) - t0) / 1e3
        dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3
        name = t["Kernel_Name"].replace("rtamd::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        print(f"{s:8.1f} {dur:8.1f}  {q(t):>3}  {name}")
        byq.setdefault(q(t), []).append((int(t["Start_Timestamp"]), int(t["End_Timestamp"])))
    for k, iv in sorted(byq.items()):
        busy = sum(e - s for s, e in iv) / 1e3
        gaps = [(iv[i + 1][0] - iv[i][1]) / 1e3 for i in range(len(iv) - 1)]
        print(f"queue {k}: {len(iv)} kernels, busy {busy:.1f} us, gaps between them " +
              ", ".join(f"{g:.1f}" for g in gaps))


if __name__ == "__main__":
    main()
