"""Summarise rocprofv3 --pmc CSVs (one row per dispatch x counter) into the mean
counter value per kernel, plus derived ratios."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")[:60]
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in vals.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    for c in sorted(m):
        print(f"   {c:34s} {m[c]:.4g}")
    if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        print("   MFMA busy / SQ busy               ", round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1, m["SQ_BUSY_CYCLES"]), 4))
    if "TCC_HIT_sum" in m:
        print("   L2 hit rate                       ", round(m["TCC_HIT_sum"] / max(1, m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4))
