#!/usr/bin/env python3
"""Phase breakdown of the resident smoothing sweeps (k_brick_sweeps) from a
GLS_SWEEP_TIMING=1 build (dealii-ns-gls_amd/lib/var/sweep_timing.so, loaded
through GLS_AMD_LIB): per sweep, workgroup lane 0's wall-clock stamps at the
sweep start, after the neighbour wait, after staging, after the cell
rounds and after the write-out (the sixth stamp is unused).  Runs a few Re3900 r0..r2
V-cycles (10 coarse sweeps) and prints medians over bricks and launches."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) < 2:
    out = os.path.join(ROOT, "gpurun_out", "sweep_timing.bin")
    if os.path.exists(out):
        os.remove(out)
    env = dict(os.environ, GLS_AMD_LIB=os.path.join(ROOT, "dealii-ns-gls_amd", "lib", "var",
                                                    "sweep_timing.so"),
               GLS_SWEEP_TIMING_OUT=out)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prof_vcycle.py"), "10"],
                       env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout.strip(), r.stderr.strip()[-500:])
    path = out
else:
    path = sys.argv[1]
raw = np.fromfile(path, dtype=np.uint64)
pos, launches = 0, []
while pos < raw.size:
    nb, ns = int(raw[pos]), int(raw[pos + 1])
    st = raw[pos + 2: pos + 2 + nb * ns * 6].astype(np.int64).reshape(nb, ns, 6)
    launches.append(st)
    pos += 2 + nb * ns * 6
print(f"{len(launches)} launches")
TICK_NS = 10.0  # s_memrealtime: 100 MHz
by_shape = {}
for st in launches[-6:]:  # the last cycles' launches (warm)
    nb, ns, _ = st.shape
    by_shape.setdefault((nb, ns), []).append(st)
for (nb, ns), L in sorted(by_shape.items()):
    st = np.concatenate([x[None] for x in L])  # [launch][brick][sweep][6]
    ph = np.diff(st[..., :5], axis=-1) * TICK_NS / 1e3  # us
    names = ["granule wait+rebuild", "stage", "rounds", "write-out"]
    print(f"bricks {nb}, sweeps {ns}, {len(L)} launches")
    for j in range(ns):
        med = np.median(ph[:, :, j, :], axis=(0, 1))
        p90 = np.percentile(ph[:, :, j, :], 90, axis=(0, 1))
        t0 = st[:, :, j, 0]
        skew = (t0.max(axis=1) - t0.min(axis=1)).mean() * TICK_NS / 1e3
        per = ""
        if j + 1 < ns:
            per = f" period {np.median(st[:, :, j + 1, 0] - st[:, :, j, 0]) * TICK_NS / 1e3:5.2f}"
        print(f"  sweep {j}: " + "  ".join(f"{n} {m:5.2f} ({p:5.2f})" for n, m, p in zip(names, med, p90))
              + f"  start skew {skew:5.2f}" + per)
    tot = (st[:, :, -1, 4].max(axis=1) - st[:, :, 0, 0].min(axis=1)).mean() * TICK_NS / 1e3
    print(f"  launch span (first start to last write-out) {tot:.1f} us")
