"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel totals and the
per-launch sequence of the last frame."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
for r in rows:
    print(f"{r['Name'][:80]:80s} calls={r['Calls']:>4} total_ms={float(r['TotalDurationNs'])/1e6:9.3f} "
          f"avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):6.2f}")
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
print("--- last launches: name, us, VGPR, scratch, LDS")
for t in tr[-n:]:
    dur = (int(t['End_Timestamp']) - int(t['Start_Timestamp'])) / 1e3
    print(f"{t['Kernel_Name'][:60]:60s} {dur:9.1f} {t['VGPR_Count']:>4} {t['Scratch_Size']:>5} {t['LDS_Block_Size']:>6}")
