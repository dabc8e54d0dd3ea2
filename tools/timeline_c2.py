"""Per-generation kernel timeline of a C2 run from a rocprofv3 kernel trace:
the kernels of a few steady-state generations (cut at k_publish_c, the last
kernel of a generation's update), each with its start offset from the
generation's start, its duration and the idle gap on the GPU before it.

    python tools/timeline_c2.py <dir with *kernel_trace.csv> [generations]
"""
import csv
import glob
import os
import re
import sys


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    return n.split("(")[0].replace("void ", "").strip()


def main():
    d = sys.argv[1]
    ngen = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in csv.DictReader(open(f))]
    rows.sort()
    cuts = [i for i, r in enumerate(rows) if r[2].endswith("k_publish_c")]
    if len(cuts) < ngen + 3:
        print("not enough generations in the trace", len(cuts))
        return
    # steady state: generations in the middle of the timed run
    mid = len(cuts) // 2
    for g in range(mid, mid + ngen):
        a, b = cuts[g] + 1, cuts[g + 1] + 1
        t0 = rows[a][0]
        busy, prev_end = 0, rows[a - 1][1]
        print(f"--- generation (publish to publish): {(rows[b - 1][1] - rows[a - 1][1]) / 1e3:.1f} us")
        for s, e, n in rows[a:b]:
            gap = s - prev_end
            print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap / 1e3:7.1f}  {n}")
            busy += e - max(s, prev_end) if e > prev_end else 0
            prev_end = max(prev_end, e)
        print(f"    GPU busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
