"""Run one C2 left pass with DSX_TIMELINE and summarise block residency (dev tool, GPU box)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402

from bench import CONFIGS  # noqa: E402

# usage: python tools/timeline.py [grid] [config]   (config of bench.py, default c2)
grid = int(sys.argv[1]) if len(sys.argv) > 1 else 0
cfg = dict(CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c2"])
H, W, D = cfg.pop("H"), cfg.pop("W"), cfg["num_disp"]
cfg.pop("desc")
L, R, _ = stereo_pair(H, W, 0, D, seed=1)
tL, tR = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
out = torch.empty((H, W), dtype=torch.int16, device="cuda")
kw = {"out_float": torch.empty((H, W), dtype=torch.float32, device="cuda")} if os.environ.get("TL_FLOAT") else {}  # bench's outputs
m = HipBlockMatcher(grid_blocks=grid, **cfg)
for _ in range(int(os.environ.get("TL_WARM", "3"))):  # TL_WARM=2000: settled clocks (steady state)
    m.compute_device(tL, tR, out_fixed=out, **kw)
torch.cuda.synchronize()
path = "/tmp/tl.bin"
os.environ["DSX_TIMELINE"] = path
m.compute_device(tL, tR, out_fixed=out, **kw)
torch.cuda.synchronize()
del os.environ["DSX_TIMELINE"]
raw = np.fromfile(path, dtype=np.uint64)
t = raw[: 4 * 65536].reshape(-1, 4)
t = t[t[:, 1] > 0]
st, en = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
t0 = st.min()
st, en = (st - t0) / 100.0, (en - t0) / 100.0  # memrealtime = 100 MHz -> us
hw = t[:, 2].astype(np.int64)
xcc = t[:, 3].astype(np.int64) & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
print(f"grid={len(t)} span={en.max():.1f}us start: min {st.min():.1f} med {np.median(st):.1f} p90 {np.percentile(st,90):.1f} max {st.max():.1f}")
print(f"dur: min {np.min(en-st):.1f} med {np.median(en-st):.1f} max {np.max(en-st):.1f}")
late = st > 0.25 * en.max()
print(f"blocks starting after 25% of span: {late.sum()}")
key = xcc * 1000 + se * 100 + sh * 16 + cu
u, c = np.unique(key, return_counts=True)
print("distinct CUs:", len(u), "blocks per CU min/med/max:", c.min(), np.median(c), c.max())
for thr in (1, 5, 10, 20, 50):
    print(f"resident at t={thr}us:", int(((st <= thr) & (en > thr)).sum()))
ext = np.fromfile(path, dtype=np.uint64).reshape(-1)
if ext.size >= 12 * 65536:
    ps = ext[4 * 65536:].reshape(-1, 8)[: len(t)]
    if ps[:, 7].sum() > 0:
        steps = ps[:, 7].astype(np.float64)
        names = ["update", "prefetch-issue", "horizontal", "barrier1", "epilogue", "store-row", "barrier2"]
        tot = ps[:, :7].astype(np.float64).sum(0) / steps.sum()
        print("cycles per row-step (s_memtime):", {n: round(v, 1) for n, v in zip(names, tot)}, "sum", round(tot.sum(), 1))
# duration by strip (block b owns strip b * NS / NG in the one-strip-per-block regime)
NS = (W + 31) // 32
dur = en - st
bs_ = np.arange(len(t))
strip = bs_ * NS // len(t)
per = [dur[strip == s].mean() for s in range(NS)]
print("mean block duration per strip (us):", " ".join(f"{v:.0f}" for v in per))
print("slowest 10 blocks (block, strip, dur, start):", [(int(b), int(strip[b]), round(float(dur[b]), 1), round(float(st[b]), 1)) for b in np.argsort(-dur)[:10]])
order = np.lexsort((bs_, key))  # blocks of each CU in dispatch (block id) order
rank = np.empty(len(t), np.int64)
ks, first = np.unique(key[order], return_index=True)
for i, f in enumerate(first):
    e = first[i + 1] if i + 1 < len(first) else len(order)
    rank[order[f:e]] = np.arange(e - f)
print("mean duration by CU-slot rank (us):", " ".join(f"{dur[rank == r].mean():.1f}" for r in range(rank.max() + 1)))
print("mean duration by XCD (us):", " ".join(f"{dur[xcc == x].mean():.1f}" for x in range(8)))
print("mean end by CU-slot rank (us):", " ".join(f"{en[rank == r].mean():.1f}" for r in range(rank.max() + 1)))
