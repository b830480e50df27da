#!/usr/bin/env python3
"""Per-V-cycle kernel attribution from scripts/prof_vcycle_trace.sh's
rocprofv3 kernel trace: the second-to-last cycle, grouped by kernel and grid."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/vtrace/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
# a cycle starts at the finest level's first relaxation (k_relax_first or,
# unfused, the copy_to_mg conversion)
g_top = max([int(r["Grid_Size_X"]) for r in rows if "k_relax_first" in r["Kernel_Name"]] or [0])
mark = [i for i, r in enumerate(rows)
        if "k_relax_first" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == g_top]
if len(mark) < 2:  # unfused finest level: the copy_to_mg conversion
    mark = [i for i, r in enumerate(rows) if "k_convert<double, float>" in r["Kernel_Name"]]
a, b = mark[-2], mark[-1]
cyc = rows[a:b]
agg, tot = {}, 0
for r in cyc:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    name = name.split("(")[0].replace("void ", "").replace("gls::", "")
    key = (name[:44], r["Grid_Size_X"])
    agg.setdefault(key, [0, 0])
    agg[key][0] += 1
    agg[key][1] += d
    tot += d
print(f"cycle wall {(int(rows[b]['Start_Timestamp']) - int(cyc[0]['Start_Timestamp'])) / 1e3:.1f} us,"
      f" kernels {tot / 1e3:.1f} us, {len(cyc)} launches")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k[0]:44s} grid {k[1]:>8s} n {v[0]:3d} total {v[1] / 1e3:8.2f} us avg {v[1] / v[0] / 1e3:6.2f}")
