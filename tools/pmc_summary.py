"""Aggregate rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv)
per kernel family over the LAST rendered frame of each pass (one bench step =
one render; the work-count frame is excluded by kernel name)."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"


def family(name):
    m = re.search(r"(wf_\w+<[^>]*>|wf_\w+|trace_frame_kernel<[^>]*>|path_kernel<[^>]*>)", name)
    return m.group(1) if m else name[:40]


tot = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
calls = collections.defaultdict(set)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        fam = family(r["Kernel_Name"])
        if "true>" in fam and fam.endswith("true>") and "wf_nearest" in fam and ", true, true" in fam:
            pass
        tot[fam][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (f, r["Dispatch_Id"])
        if key not in calls[fam]:
            calls[fam].add(key)
            dur[fam] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
names = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
         "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU",
         "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE", "FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"]
for fam in sorted(tot, key=lambda k: -dur[k]):
    c = tot[fam]
    print(f"== {fam}  (summed over all passes' dispatches: {len(calls[fam])} dispatches, {dur[fam]:.2f} ms)")
    line = "  ".join(f"{n}={c[n]:.3g}" for n in names if n in c)
    print("   " + line)
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        print(f"   valu-active/wave-cycles={c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}  wait_any/wave-cycles="
              f"{c.get('SQ_WAIT_ANY', 0) / wc:.3f}  wait_inst/wave-cycles={c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}")
    if c.get("SQ_INSTS_VALU") and c.get("SQ_WAVES"):
        print(f"   valu insts per wave={c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}  vmem rd per wave="
              f"{c.get('SQ_INSTS_VMEM_RD', 0) / c['SQ_WAVES']:.0f}")
    if c.get("TCC_HIT_sum") or c.get("TCC_MISS_sum"):
        h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        print(f"   L2 hit rate={h / max(1.0, h + m):.3f}  (hits {h:.3g}, misses {m:.3g})")
    if c.get("TCP_TOTAL_CACHE_ACCESSES_sum") and c.get("TCP_TCC_READ_REQ_sum") is not None:
        print(f"   L1 accesses={c['TCP_TOTAL_CACHE_ACCESSES_sum']:.3g}  L1->L2 read requests={c['TCP_TCC_READ_REQ_sum']:.3g}")
