"""Per-kernel durations (us) of the last hole-filling call in a rocprofv3 kernel trace (dev tool)."""
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[-1]
rows = [r for r in csv.DictReader(open(f)) if "tl_" in r["Kernel_Name"] or "memset" in r["Kernel_Name"].lower()]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "tl_init" in r["Kernel_Name"]]
seq = rows[starts[-1]:]
t0 = int(seq[0]["Start_Timestamp"])
tot = 0
for r in seq:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f'{(int(r["Start_Timestamp"]) - t0) / 1e3:8.1f} {d:7.1f} {r["Kernel_Name"][:60]}')
print("sum", round(tot, 1), "span", (int(seq[-1]["End_Timestamp"]) - t0) / 1e3)
