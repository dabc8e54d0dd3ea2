"""Summarise a rocprofv3 MFMA counter pass (SQ_VALU_MFMA_BUSY_CYCLES,
SQ_INSTS_VALU_MFMA_MOPS_F64, GRBM_GUI_ACTIVE in one run) per kernel:
average per dispatch, the FP64 MFMA work (one MOP = 512 FLOP: a
v_mfma_f64_16x16x4f64 is 4 MOPs = 2048 FLOP), the clock (GRBM_GUI_ACTIVE is
summed over the 8 XCDs) and the MFMA-busy fraction over the chip's 1024
SIMDs for the dispatch's duration.

    python tools/pmc_mfma_summary.py <pmc dir> [kernel substring ...] > out.csv
"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
keys = sys.argv[2:] or ["k_rankmu_tile"]
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(dict)
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"]
    k = next((k for k in keys if k in name), None)
    if k is None:
        continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
w = csv.writer(sys.stdout)
w.writerow(["kernel", "dispatches", "avg_us", "mfma_busy_cycles", "mfma_mops_f64", "mfma_gflop", "grbm_gui_active",
            "clock_ghz", "mfma_busy_frac", "mfma_tflops"])
for k, c in acc.items():
    n = len(dur[k])
    t = sum(dur[k].values()) / n
    busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(c["SQ_VALU_MFMA_BUSY_CYCLES"])
    mops = sum(c["SQ_INSTS_VALU_MFMA_MOPS_F64"]) / len(c["SQ_INSTS_VALU_MFMA_MOPS_F64"])
    gui = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"])
    cyc = gui / 8.0
    w.writerow([k, n, round(t * 1e6, 2), int(busy), int(mops), round(mops * 512 / 1e9, 4), int(gui),
                round(cyc / t / 1e9, 3), round(busy / (1024 * cyc), 4), round(mops * 512 / t / 1e12, 2)])
