#!/usr/bin/env python3
"""Overlap of the ghost exchange with the brick kernels in a kernel trace of
threaded in-process group vmults (scripts/prof_dist_threaded.py under
rocprofv3 --kernel-trace): the exchange copies run as blit kernels
(__amd_rocclr_copyBuffer) on each member's communication stream; reports how
much of their time falls inside a k_brick of the same or another member, per
stream and in total, and one vmult's launch timeline.
    python scripts/dist_overlap.py gpurun_out/r5h/trace/run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"],
           r["Queue_Id"]) for r in rows]
    ks.sort()
    brick = [(a, b) for a, b, n, *_ in ks if "k_brick" in n]
    copies = [(a, b, st) for a, b, n, st, _ in ks if "copyBuffer" in n]
    # the timed vmults: copies after the setup (the last 2 x reps x peers copies)
    t_tot = t_ov = 0
    per = defaultdict(lambda: [0, 0])
    for a, b, st in copies:
        ov = 0
        for x, y in brick:
            lo, hi = max(a, x), min(b, y)
            if hi > lo:
                ov += hi - lo
        ov = min(ov, b - a)
        t_tot += b - a
        t_ov += ov
        per[st][0] += b - a
        per[st][1] += ov
    print(f"{len(copies)} exchange copies, {len(brick)} brick kernels")
    print(f"copy time {t_tot / 1e3:.1f} us, inside a brick kernel {t_ov / 1e3:.1f} us "
          f"({100 * t_ov / max(t_tot, 1):.0f} %)")
    for st, (a, b) in sorted(per.items()):
        print(f"  stream {st}: copies {a / 1e3:.1f} us, overlapped {b / 1e3:.1f} us")
    # the last vmult pair: launches in time order (relative us)
    tail = ks[-24:]
    t0 = tail[0][0]
    print("last launches (start..end us, stream, kernel):")
    for a, b, n, st, q in tail:
        print(f"  {(a - t0) / 1e3:8.1f} .. {(b - t0) / 1e3:8.1f}  s{st} q{q}  {n[:70]}")


if __name__ == "__main__":
    main(sys.argv[1])
