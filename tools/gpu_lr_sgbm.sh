#!/bin/bash
# OpenCV's LR form on the fused pass: its GPU tests + the full-size config and parity suites, a same-box
# A/B of the headline configs against tools/explib/libdsx_base.so, and bm-vs-sgbm LR kernel times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_sgbm_lr.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/lr_sgbm_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/lr_sgbm_tests.txt; [ $rc -eq 0 ] || exit $rc
CONFIGS="c2 c2r c4" REPS=2 STEPS=1000 bash tools/lib_ab.sh lr_sgbm_ab tools/explib/libdsx_base.so
for lf in sgbm; do
python3 - <<'PY'
import torch, time, json, sys
sys.path.insert(0, '.')
from depthestimation_amd.matcher import HipBlockMatcher
from depthestimation_amd.synthetic import stereo_pair
from depthestimation_amd.configs import CONFIGS
for c in ("c2r", "c4"):
    cfg = CONFIGS[c]; H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
    L, R, _ = stereo_pair(H, W, 0, D, seed=1234)
    dL, dR = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    out = torch.empty((H, W), dtype=torch.int16, device="cuda")
    res = {}
    for form in ("bm", "sgbm"):
        m = HipBlockMatcher(num_disp=D, block_size=cfg["block_size"], uniqueness_ratio=10, disp12_max_diff=1, lr_form=form, timing=True)
        for _ in range(300): m.compute_device(dL, dR, out_fixed=out)
        torch.cuda.synchronize(); m.reset_times()
        for _ in range(300): m.compute_device(dL, dR, out_fixed=out)
        torch.cuda.synchronize()
        res[form] = {k: round(v[0]*1e3, 2) for k, v in m.kernel_times().items()}
        m.close()
    print(json.dumps({"config": c, "us": res}))
PY
done
