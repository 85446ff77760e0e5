"""Turn a tools/prof.sh output dir (gpurun_out/prof_<tag>) into committed summaries under profiles/:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.txt            per-kernel average PMC values per dispatch
  profiles/traffic.json             {"<config>:<path>:<kernel>": {"hbm_bytes_per_launch": ...}}
  profiles/valu_counts.json         {"<config>:<path>:<kernel>": {"SQ_INSTS_VALU": ...}} (VALU roofline)
HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE/WRITE_SIZE are KiB from separate
--pmc passes; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so it is doubled
(exact for K2's 16-B streaming reads; an upper bound for the fused pass's 4-B row loads).

usage: python tools/make_profiles.py <prof dir> <tag> <config> <path>
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

# kernel names: vol_wta / lr_fixup by name, bm2<R, SSD, NW, SIDE[, ABS]> by its SIDE argument
SIDES = {"0": "bm_pass_left", "3": "bm_pass_left", "4": "bm_pass_left", "1": "bm_pass_right", "2": "cost_volume"}


def short(k):
    if "vol_wta" in k:
        return "volume_wta"
    if "lr_fixup_sgbm" in k:
        return "lr_fixup_sgbm"
    if "lr_fixup" in k:
        return "lr_fixup"
    if "spk_tile" in k:
        return "speckle_tile"
    if "post_tail3" in k:
        return "post_tail"
    m = re.search(r"bm2<\s*\d+,\s*\w+,\s*\d+,\s*(\d)", k)
    return SIDES[m.group(1)] if m else k


def main(src, tag, config, path):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))[0]
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    avg_ns = {r["Name"]: float(r["AverageNs"]) for r in rows}
    calls = {r["Name"]: int(r["Calls"]) for r in rows}
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = [f"# rocprofv3 PMC, average per dispatch ({tag}; {config}, path={path})",
             "# FETCH_SIZE / WRITE_SIZE in KiB; separate --pmc passes per counter group (tools/prof.sh)"]
    tp = os.path.join(prof, "traffic.json")
    traffic = json.load(open(tp)) if os.path.exists(tp) else {}
    vp = os.path.join(prof, "valu_counts.json")
    valu = json.load(open(vp)) if os.path.exists(vp) else {}
    # kernels that share a short name (e.g. a secondary leg's matcher next to the config's own) are
    # listed each, and the entry of traffic.json / valu_counts.json is the most dispatched one's
    for k, cs in sorted(acc.items(), key=lambda kv: calls.get(kv[0], 0)):
        if "rocclr" in k or "dsx::" not in k:  # torch fill kernels of the bench harness
            continue
        lines.append(f"{k}  [{short(k)}]  avg_ns={avg_ns.get(k)}")
        for c, v in sorted(cs.items()):
            lines.append(f"    {c:28s} {sum(v) / len(v):18.1f}")
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            rd = 2 * m["FETCH_SIZE"] * 1024
            wr = m["WRITE_SIZE"] * 1024
            traffic[f"{config}:{path}:{short(k)}"] = {
                "hbm_bytes_per_launch": round(rd + wr), "read_bytes": round(rd), "write_bytes": round(wr),
                "avg_ns": avg_ns.get(k), "source": f"profiles/{tag}_pmc.txt (2*FETCH_SIZE + WRITE_SIZE, KiB->B)"}
            lines.append(f"    => HBM bytes/launch (2*FETCH + WRITE) {rd + wr:,.0f}")
        if "SQ_INSTS_VALU" in m:
            e = {"SQ_INSTS_VALU": round(m["SQ_INSTS_VALU"]), "avg_ns": avg_ns.get(k),
                 "source": f"profiles/{tag}_pmc.txt (rocprofv3 --pmc, average per dispatch)"}
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_THREAD_CYCLES_VALU", "GRBM_GUI_ACTIVE"):
                if c in m:
                    e[c] = round(m[c])
            valu[f"{config}:{path}:{short(k)}"] = e
        if "SQ_WAVE_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
            lines.append(f"    => VALU instr/wave {m.get('SQ_INSTS_VALU', 0) / max(m.get('SQ_WAVES', 1), 1):,.0f}; "
                         f"wait_any/wave_cycles {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.2f}")
    open(os.path.join(prof, f"{tag}_pmc.txt"), "w").write("\n".join(lines) + "\n")
    json.dump(traffic, open(tp, "w"), indent=1, sort_keys=True)
    json.dump(valu, open(vp, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:5])
