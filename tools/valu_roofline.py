"""VALU-issue roofline of the fused block-matching pass (SURVEY.md 8(d) D2 for a kernel that is
bound by VALU issue, not HBM; VERDICT r1 "make the headline roofline true").

The fused pass keeps the cost volume in LDS, so its HBM traffic is ~6-16 B/px and HBM is not its
bound. Its bound is vector-instruction issue: every SIMD can issue one VALU wave-instruction at a
time, and each form occupies the SIMD for a measured number of cycles (tools/ubench3.hip, table in
profiles/issue_costs.json: v_add_u32 / v_add_f32 / v_fma_f32 ~2.3 cycles, v_pk_* / v_max* /
v_perm ~4.1, ...).  For a launch that executes N VALU wave-instructions (rocprofv3 SQ_INSTS_VALU)
whose issue-cost-weighted mean is c cycles, the issue work is N * c SIMD-cycles, and the chip
offers 1024 SIMDs * f_clk SIMD-cycles per second, so

    frac = N * c / (1024 * f_clk * t_kernel)          (1.0 = every SIMD issuing VALU all the time)

c is the mean issue cost over the kernel's row loop (the loop that executes once per (strip, row)
step and holds >95 % of the dynamic VALU count), read from the compiled code object's assembly.

usage:
  python tools/valu_roofline.py mix   <kernel .s> <symbol substring> [--costs profiles/issue_costs.json]
  python tools/valu_roofline.py frac  <pmc.txt> <mix.json key> <t_kernel_ns> [--clock-ghz 2.4]
  python tools/valu_roofline.py build                      (writes profiles/valu_mix.json for the
                                                            bench instantiations, from a fresh -S build)
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COSTS = os.path.join(ROOT, "profiles", "issue_costs.json")
MIX = os.path.join(ROOT, "profiles", "valu_mix.json")
N_SIMD = 1024  # 256 CUs x 4 SIMDs (MI355X)

# the instantiations bench.py runs (BASELINE configs, fused path): (radius, SSD, NW, SIDE)
# (radius, SSD layout, NW, SIDE, ABS): ABS = SAD in the one-disparity-per-lane u32 layout (BM_SAD1, D <= 64)
BENCH_KERNELS = {
    "c1": (2, True, 1, 0, True), "c2": (4, False, 1, 0, False), "c3": (5, True, 4, 3, False),
    "c4": (2, False, 1, 3, False), "c5": (7, False, 2, 0, False), "c2r": (4, False, 1, 3, False),
}


def symbol(r, ssd, nw, side, abs_=False):
    return f"_ZN3dsx3bm2ILi{r}ELb{int(ssd)}ELi{nw}ELi{side}ELb{int(abs_)}EEEvNS_7Bm2ArgsE"


def kernel_label(r, ssd, nw, side, abs_=False):
    return f"bm2<R={r},{'SAD1' if abs_ else ('SSD' if ssd else 'SAD')},NW={nw},SIDE={side}>"


def base_op(op: str) -> str:
    """v_add_u32_e32 / _e64 / _sdwa / _dpp -> v_add_u32 (the encoding does not change the issue slot)."""
    return re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)


def function_body(asm: str, sym: str) -> str:
    m = re.search(r"\n" + re.escape(sym) + r":[^\n]*\n(.*?)\.Lfunc_end", asm, re.S)
    if not m:
        raise SystemExit(f"symbol {sym} not in the assembly")
    return m.group(1)


def blocks(body: str):
    """[(label, [ops], branch targets)] in layout order."""
    out = []
    for b in re.split(r"\n(?=\.LBB\d+_\d+:)", body):
        lab = b.split(":")[0] if b.startswith(".LBB") else "entry"
        ops, targets = [], []
        for line in b.split("\n"):
            if not line.startswith("\t"):
                continue
            t = line.strip()
            if not t or t.startswith((".", ";")):
                continue
            op = t.split()[0]
            ops.append(op)
            if op.startswith(("s_cbranch", "s_branch")):
                mt = re.search(r"(\.LBB\d+_\d+)", t)
                if mt:
                    targets.append(mt.group(1))
        out.append((lab, ops, targets))
    return out


def row_loops(bl, min_valu=150, share=0.5):
    """The per-row loop bodies, from back edges (a branch to an earlier label) as block index
    ranges: drop loops that contain two disjoint loops of >= min_valu VALU ops (the segment loop
    around the FAST and clamped copies of the row loop), merge the overlapping rest into clusters
    (a rotated loop has several latches), and keep the clusters holding >= share of the largest
    one's VALU ops (the row loop of each segment copy; the (2R+1)-row init loop and the rare
    padding / invalid-band loops fall below)."""
    index = {lab: i for i, (lab, _, _) in enumerate(bl)}
    loops = set()
    for j, (_, _, tg) in enumerate(bl):
        for t in tg:
            i = index.get(t)
            if i is not None and i <= j:
                loops.add((i, j))

    def nvalu(rng):
        return sum(1 for k in range(rng[0], rng[1] + 1) for o in bl[k][1] if o.startswith("v_"))

    heavy = sorted(lp for lp in loops if nvalu(lp) >= min_valu)

    def is_parent(lp):
        inner = [o for o in heavy if o != lp and lp[0] <= o[0] and o[1] <= lp[1]]
        return any(a[1] < b[0] or b[1] < a[0] for a in inner for b in inner)

    cand = [lp for lp in heavy if not is_parent(lp)]
    clusters = []
    for lp in sorted(cand):
        if clusters and lp[0] <= clusters[-1][1]:
            clusters[-1] = (clusters[-1][0], max(clusters[-1][1], lp[1]))
        else:
            clusters.append(lp)
    if not clusters:
        return [], nvalu
    top = max(nvalu(c) for c in clusters)
    return [c for c in clusters if nvalu(c) >= share * top], nvalu


def loop_mix(asm_path: str, sym: str):
    bl = blocks(function_body(open(asm_path).read(), sym))
    loops, nvalu = row_loops(bl)
    if not loops:
        raise SystemExit(f"{sym}: no row loop found")
    mix = Counter()
    for i, j in loops:
        for k in range(i, j + 1):
            mix.update(base_op(o) for o in bl[k][1] if o.startswith("v_"))
    return mix, [(bl[i][0], bl[j][0], nvalu((i, j))) for i, j in loops]


def weigh(mix: Counter, costs: dict, families: dict | None = None):
    """Mean issue cost of a VALU mix; a form without a measured cost takes its family's (v_cmp_*,
    v_pk_*, ...) or else the table's default (the 4-cycle class) and is reported as unpriced."""
    default = costs["_default"]
    total = n = 0.0
    unpriced = Counter()
    for op, k in mix.items():
        c = costs.get(op)
        if c is None:
            c = next((v for p, v in (families or {}).items() if op.startswith(p)), None)
            if c is not None:
                total += c * k
                n += k
                continue
            unpriced[op] += k
            c = default
        total += c * k
        n += k
    return total / n, unpriced


def cmd_mix(asm, sub, costs_path=COSTS):
    table = json.load(open(costs_path))
    costs, fam = table["cycles"], table.get("families")
    asm_text = open(asm).read()
    syms = [s for s in re.findall(r"\n(_Z\w+):", asm_text) if sub in s]
    for s in syms:
        mix, loops = loop_mix(asm, s)
        c, unpriced = weigh(mix, costs, fam)
        print(s, "loops", loops, f"mean issue cost {c:.3f} cycles over {sum(mix.values())} VALU ops")
        for op, k in mix.most_common(40):
            print(f"   {op:28s} {k:6d}  {costs.get(op, '?')}")
        if unpriced:
            print("   unpriced:", dict(unpriced))


def cmd_build():
    """-S build of the radius TUs the bench kernels live in, mean issue cost per bench kernel."""
    table = json.load(open(COSTS))
    costs, fam = table["cycles"], table.get("families")
    src = os.path.join(ROOT, "depthestimation_amd", "csrc", "dsx_bm.hip")
    tmp = os.path.join("/tmp", "dsx_valu_mix")
    os.makedirs(tmp, exist_ok=True)
    out = {}
    for name, (r, ssd, nw, side, abs_) in BENCH_KERNELS.items():
        s_path = os.path.join(tmp, f"r{r}.s")
        if not os.path.exists(s_path) or os.path.getmtime(s_path) < os.path.getmtime(src):
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-DDSX_RADIUS={r}",
                            "--cuda-device-only", "-S", "-o", s_path, src], check=True)
        sym = symbol(r, ssd, nw, side, abs_)
        mix, loops = loop_mix(s_path, sym)
        c, unpriced = weigh(mix, costs, fam)
        out[name] = {"kernel": kernel_label(r, ssd, nw, side, abs_), "symbol": sym,
                     "mean_issue_cycles": round(c, 4), "loop_valu_ops": sum(mix.values()),
                     "loops": [list(x) for x in loops],
                     "unpriced_ops": dict(unpriced),
                     "top_ops": dict(mix.most_common(12))}
        print(name, out[name]["kernel"], f"c = {c:.3f}", "unpriced", dict(unpriced))
    out["_source"] = ("tools/valu_roofline.py build: row-loop VALU mix of the hipcc -S code object, priced with "
                      "profiles/issue_costs.json")
    json.dump(out, open(MIX, "w"), indent=1, sort_keys=True)
    print("wrote", MIX)


def pmc_value(pmc_path: str, counter: str, kernel_pat: str = "bm_pass_left"):
    cur = None
    for line in open(pmc_path):
        if not line.startswith(" ") and f"[{kernel_pat}]" in line:
            cur = True
            continue
        if not line.startswith(" "):
            cur = None
        if cur and line.split() and line.split()[0] == counter:
            return float(line.split()[1])
    return None


def valu_frac(n_valu: float, mean_cycles: float, t_ns: float, clock_ghz: float = 2.4):
    """(achieved G wave-instr/s, peak G wave-instr/s for this mix, frac)."""
    achieved = n_valu / (t_ns * 1e-9) / 1e9
    peak = N_SIMD * clock_ghz / mean_cycles
    return achieved, peak, achieved / peak


def cmd_frac(pmc, key, t_ns, clock=2.4):
    n = pmc_value(pmc, "SQ_INSTS_VALU")
    c = json.load(open(MIX))[key]["mean_issue_cycles"]
    a, p, f = valu_frac(n, c, float(t_ns), clock)
    print(json.dumps({"SQ_INSTS_VALU": n, "mean_issue_cycles": c, "t_kernel_ns": float(t_ns), "clock_ghz": clock,
                      "achieved_Ginst_s": round(a, 2), "peak_Ginst_s": round(p, 2), "frac": round(f, 4)}))


if __name__ == "__main__":
    a = sys.argv[1:]
    if not a:
        raise SystemExit(__doc__)
    if a[0] == "mix":
        cmd_mix(a[1], a[2], *(a[4:5] if len(a) > 4 else []))
    elif a[0] == "build":
        cmd_build()
    elif a[0] == "frac":
        clock = float(a[a.index("--clock-ghz") + 1]) if "--clock-ghz" in a else 2.4
        cmd_frac(a[1], a[2], a[3], clock)
    else:
        raise SystemExit(__doc__)
