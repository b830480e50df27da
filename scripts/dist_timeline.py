#!/usr/bin/env python3
"""Phase order of the last partitioned vmult in a rocprofv3 kernel +
memory-copy trace of scripts/prof_dist_group.py (one line per dispatch /
copy: start offset, duration, name, grid)."""
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dist_trace"
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gls::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:60],
                     r.get("Grid_Size_X", "")))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     "memcpy " + r.get("Direction", ""), r.get("Size", "")))
rows.sort()
# the last vmult: from its first k_pack (every member that sends packs) on
packs = [i for i, r in enumerate(rows) if r[2].startswith("k_pack")]
start = packs[-1]
while start > 0 and rows[start - 1][2].startswith("k_pack"):
    start -= 1
t0 = rows[start][0]
for s, e, name, grid in rows[start:]:
    print(f"{(s - t0) / 1e3:8.2f} us  {(e - s) / 1e3:7.2f} us  {name:60s} {grid}")
