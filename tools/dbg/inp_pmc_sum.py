"""Per-step counters of the last hole fill in inp_pmc.sh's passes (dev)."""
import csv, glob, sys, collections
rows = collections.defaultdict(dict)
for f in sorted(glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True)):
    recs = [r for r in csv.DictReader(open(f)) if "tl_" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in recs})
    # the last fill: from the last tl_init on
    inits = sorted({int(r["Dispatch_Id"]) for r in recs if "tl_init" in r["Kernel_Name"]})
    ids = [d for d in ids if d >= inits[-1]]
    for k, d in enumerate(ids):
        for r in recs:
            if int(r["Dispatch_Id"]) == d:
                rows[k][r["Counter_Name"]] = rows[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
                rows[k]["kernel"] = r["Kernel_Name"][:30]
names = sorted({n for v in rows.values() for n in v if n != "kernel"})
print("step " + " ".join(f"{n[:14]:>14}" for n in names))
for k in sorted(rows):
    print(f"{k:4d} " + " ".join(f"{rows[k].get(n, 0):14.0f}" for n in names) + " " + rows[k].get("kernel", ""))
