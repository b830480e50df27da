#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/.../run_counter_collection.csv):
per-kernel mean of every counter, and the HBM traffic per launch of the
vmult kernels (FETCH_SIZE x2 gfx950 wide-read correction + WRITE_SIZE, KiB)."""
import csv, glob, json, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for (k, c), v in sorted(agg.items()):
    out.setdefault(k, {})[c] = sum(v) / len(v)
traffic = 0.0
prec_t = "double" if (sys.argv[3] if len(sys.argv) > 3 else "f64") == "f64" else "float"
for k, d in out.items():
    # the headline precision only (bench's parity check also runs the FP32
    # level operator under the same passes)
    if ("k_brick" in k or "k_shared_reduce" in k) and prec_t in k:
        traffic += 1024 * (2 * d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0))
for k, d in out.items():
    print(k)
    for c, v in d.items():
        print(f"   {c:24s} {v:16.1f}")
wl = {"nref": int(sys.argv[2]) if len(sys.argv) > 2 else 2,
      "precision": sys.argv[3] if len(sys.argv) > 3 else "f64"}
res = {"bytes_per_launch": traffic, "workload": wl,
       "method": "per vmult: k_brick + k_shared_reduce, 1024*(2*FETCH_SIZE + WRITE_SIZE) "
                 "(gfx950: FETCH_SIZE counts half of wide coalesced reads)",
       "counters": out}
json.dump(res, open(f"{root}/traffic.json", "w"), indent=1)
print("traffic bytes per vmult:", traffic)
