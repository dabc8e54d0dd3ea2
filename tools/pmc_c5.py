"""Summarise the C5 FETCH_SIZE / WRITE_SIZE passes for the rollout-forward
launches of k_vr_gemm<1> (4096 rows: the largest Grid_Size among its
dispatches; the update's launches are smaller), the bench's `roofline` kernel; FETCH_SIZE x2 per the gfx950 correction
(MI355X_MICROARCH.md, HBM/rocprofv3 section).

    python tools/pmc_c5.py <pmc_fetch dir> <pmc_write dir> > profiles/r2/c5_pmc_traffic.csv
"""
import csv
import glob
import os
import sys


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter and "k_vr_gemm<1>" in r["Kernel_Name"]]
    grid = max(int(r["Grid_Size"]) for r in rows)
    return [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == grid]


def main():
    f, w = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    wr = csv.writer(sys.stdout)
    wr.writerow(["kernel", "dispatches", "fetch_KB_raw", "fetch_KB_x2", "write_KB"])
    fa, wa = sum(f) / len(f), sum(w) / len(w)
    wr.writerow(["kg::vr::k_vr_gemm<1> (rollout, 4096x256x256)", len(f), f"{fa:.1f}", f"{2 * fa:.1f}", f"{wa:.1f}"])


if __name__ == "__main__":
    main()
