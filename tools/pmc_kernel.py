"""Average of every PMC counter over the dispatches of kernels whose name
contains a pattern (rocprofv3 --pmc ... --output-format csv directory).

    python tools/pmc_kernel.py <dir> <pattern>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d, pat = sys.argv[1], sys.argv[2]
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            name = r["Kernel_Name"].split("(")[0][-50:]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, ctrs in acc.items():
        print(name)
        for c, v in sorted(ctrs.items()):
            print(f"  {c:28s} n={len(v):4d} avg={sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main()
