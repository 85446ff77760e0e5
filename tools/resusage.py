"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel
(VGPRs, AGPRs, VGPR spills, SGPR spills, occupancy, LDS).  Usage:
    hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/resusage.py [filter]"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"),
                     ("sspill", r"SGPRs Spill: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f"{r['name']:<48} vgpr {r.get('vgpr', '?'):>4} agpr {r.get('agpr', '?'):>3} vspill {r.get('vspill', '?'):>3} "
              f"sspill {r.get('sspill', '?'):>4} occ {r.get('occ', '?')} lds {r.get('lds', '?')}")
