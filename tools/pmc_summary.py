"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs)
into per-kernel average KB per dispatch.

FETCH_SIZE on gfx950 counts 128-B fabric read requests at 64 B
(MI355X_MICROARCH.md, HBM/rocprofv3 section): `fetch_KB_x2` applies that x2
correction (exact for wide coalesced streaming reads; an upper estimate for
the 8-B/lane reads these FP64 kernels mostly issue).  WRITE_SIZE is exact.

    python tools/pmc_summary.py <pmc_fetch dir> <pmc_write dir> > out.csv
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = n.split("(")[0].replace("void ", "").strip()
    return n


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "dispatches", "fetch_KB_raw", "fetch_KB_x2", "write_KB"])
    for k in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0]))):
        f, wr = fetch.get(k, []), write.get(k, [])
        fa = sum(f) / len(f) if f else float("nan")
        wa = sum(wr) / len(wr) if wr else float("nan")
        w.writerow([k, max(len(f), len(wr)), f"{fa:.1f}", f"{2 * fa:.1f}", f"{wa:.1f}"])


if __name__ == "__main__":
    main()
