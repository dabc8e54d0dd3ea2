"""Summarise C5 FETCH_SIZE / WRITE_SIZE passes over every kernel of the
VRACER policy update (and the rollout), per kernel and grid: average KB per
dispatch (FETCH_SIZE x2 per the gfx950 correction, MI355X_MICROARCH.md
HBM/rocprofv3 section; WRITE_SIZE exact).

    python tools/pmc_c5_update.py <pmc_fetch dir> <pmc_write dir> > profiles/r5/c5_pmc_update_traffic.csv
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    return n.split("(")[0].replace("void ", "").strip()


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter and "k_vr_" in r["Kernel_Name"]:
            acc[(short(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return acc


def main():
    f, w = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    out = csv.writer(sys.stdout)
    out.writerow(["kernel", "grid_size", "dispatches", "fetch_KB_raw", "fetch_KB_x2", "write_KB"])
    for k in sorted(f, key=lambda k: -len(f[k])):
        fa = sum(f[k]) / len(f[k])
        wv = w.get(k, [])
        wa = sum(wv) / len(wv) if wv else float("nan")
        out.writerow([k[0], k[1], len(f[k]), f"{fa:.1f}", f"{2 * fa:.1f}", f"{wa:.1f}"])


if __name__ == "__main__":
    main()
