"""HBM bytes per render from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Each pass ran `bench.py --steps S --warmup W` (W + S uninstrumented renders,
then one RT_COUNT_WORK render, then the PCIe-inclusive rt_render calls).
Frames are split at the generation-0 wf_nearest launch; the last frame before
the RT_COUNT_WORK render (a timed-loop frame) is used.
MI355X_MICROARCH.md ("HBM"): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so it is doubled.

    python tools/pmc_traffic.py gpurun_out/pmc KEY [out.json] [chunks]

A frame rendered as several wavefront chunks (C5: 7) starts a generation-0
launch per chunk: `chunks` sums the last that many chunk-frames into one.
"""
import collections
import csv
import glob
import json
import re
import sys


def targs(name):
    return [a.strip() for a in name.split("<", 1)[1].split(">")[0].split(",")] if "<" in name else []


def family(name):
    fam = re.search(r"(wf_[a-z]+)", name).group(1)
    if fam == "wf_nearest" and targs(name)[1:2] == ["true"]:
        return "wf_camera"                       # generation 0 (kCam)
    return fam


def frames(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "wf_nearest<" in name and targs(name)[1:2] == ["true"]:      # a frame starts at generation 0
            cur = {"instrumented": targs(name)[2] == "true", "kernels": collections.defaultdict(float)}
            out.append(cur)
        if cur is None or "wf_" not in name:
            continue
        cur["kernels"][family(name)] += float(r["Counter_Value"]) * 1024.0
    # the timed loop's frames: those before the RT_COUNT_WORK render (the PCIe-inclusive
    # rt_render calls that follow it run the sparse host copies' extra kernels)
    first_inst = next((i for i, f in enumerate(out) if f["instrumented"]), len(out))
    return [f for f in out[:first_inst] if not f["instrumented"]]


def main():
    root, key = sys.argv[1], sys.argv[2]
    out_path = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    chunks = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    per = {}
    for counter, scale in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        for f in sorted(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True)):
            fr = frames(f, counter)
            if len(fr) >= chunks:
                acc = collections.defaultdict(float)
                for f_ in fr[-chunks:]:
                    for k, v in f_["kernels"].items():
                        acc[k] += v * scale
                per[counter] = dict(acc)
                break
    if len(per) != 2:
        sys.exit("need one FETCH_SIZE and one WRITE_SIZE pass")
    fams = sorted(set(per["FETCH_SIZE"]) | set(per["WRITE_SIZE"]))
    kernels = {k: {"read_bytes": per["FETCH_SIZE"].get(k, 0.0), "write_bytes": per["WRITE_SIZE"].get(k, 0.0)}
               for k in fams}
    total = sum(v["read_bytes"] + v["write_bytes"] for v in kernels.values())
    try:
        doc = json.load(open(out_path))
    except Exception:
        doc = {}
    import os
    sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rust-raytrace_amd")]
    import libraytrace
    doc[key] = {"hbm_bytes_per_launch": total, "launch": "one render (all wavefront launches of one frame)",
                "sources_id": libraytrace.sources_id(), "tuning": os.environ.get("RT_TUNE", ""),
                "per_kernel_family": kernels,
                "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, --kernel-trace only; "
                          "KiB -> bytes; FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md HBM section); "
                          "last timed-loop frame of each pass (before the RT_COUNT_WORK render)" +
                          (f" ({chunks} wavefront chunks summed)" if chunks > 1 else "")}
    json.dump(doc, open(out_path, "w"), indent=1)
    print(json.dumps(doc[key], indent=1))


if __name__ == "__main__":
    main()
