"""All kernels of the last hole-filling call in a rocprofv3 kernel trace, in order (dev tool)."""
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[-1]
rows = [r for r in csv.DictReader(open(f))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "lc_init" in r["Kernel_Name"] or "tl_init" in r["Kernel_Name"]]
seq = rows[starts[-2] if "lc_init" in rows[starts[-2]]["Kernel_Name"] else starts[-1]:]
t0 = int(seq[0]["Start_Timestamp"])
for r in seq[:40]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f'{(int(r["Start_Timestamp"]) - t0) / 1e3:8.1f} {d:7.1f} {r["Kernel_Name"][:70]}')
