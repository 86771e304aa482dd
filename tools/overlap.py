#!/usr/bin/env python3
"""Stream overlap in a rocprofv3 kernel trace of a multi-stream bench run:
over the middle steps, the fraction of wall time with >= 1 kernel running,
the time-weighted number of kernels in flight, and per kernel name the summed
duration and the part of it that ran alone (no other kernel in flight).
    python3 tools/overlap.py gpurun_out/ovl
"""
import csv
import glob
import sys
from collections import defaultdict


def main(path):
    if not path.endswith(".csv"):
        path = glob.glob(path + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    stems = [i for i, r in enumerate(rows) if "stem_" in r["Kernel_Name"]]
    # the middle third of the run (steady state, both streams busy)
    s, e = stems[len(stems) // 3], stems[2 * len(stems) // 3]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:60]) for r in rows[s:e]]
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    ev = sorted([(a, 1, n) for a, b, n in ks] + [(b, -1, n) for a, b, n in ks])
    alive, last, busy, weighted = 0, t0, 0, 0
    running = defaultdict(int)
    alone = defaultdict(int)
    total = defaultdict(int)
    for a, b, n in ks:
        total[n] += b - a
    for t, d, n in ev:
        if alive > 0:
            busy += t - last
            weighted += alive * (t - last)
        if alive == 1:
            only = [k for k, v in running.items() if v > 0][0]
            alone[only] += t - last
        last = t
        alive += d
        running[n] += d
    span = t1 - t0
    print(f"span {span / 1000:.1f} us over {len(stems[len(stems) // 3:2 * len(stems) // 3])} stem launches; "
          f"busy {busy / span:.3f}; mean kernels in flight while busy {weighted / max(busy, 1):.2f}")
    for n in sorted(total, key=lambda k: -total[k])[:25]:
        print(f"{total[n] / 1000:9.1f} us total  {alone[n] / 1000:8.1f} alone  {n}")


if __name__ == "__main__":
    main(sys.argv[1])
