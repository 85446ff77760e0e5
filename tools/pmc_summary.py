"""Summarise rocprofv3 PMC CSVs: per kernel, average counter value per dispatch (dev tool)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
meta = {}
for f in sorted(glob.glob(os.path.join(root, "pmc*", "*counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        meta[k] = (row["VGPR_Count"], row["SGPR_Count"], row["LDS_Block_Size"], row["Grid_Size"], row["Workgroup_Size"])
stats = {}
tr = glob.glob(os.path.join(root, "trace", "*kernel_stats.csv"))
if tr:
    for row in csv.DictReader(open(tr[0])):
        stats[row["Name"]] = float(row["AverageNs"])
for k, cs in acc.items():
    if "rocclr" in k:
        continue
    print(k, "vgpr/sgpr/lds/grid/wg =", meta[k], "avg_ns =", stats.get(k))
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):18.1f}")
