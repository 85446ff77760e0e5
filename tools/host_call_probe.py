"""Host cost of one HipBlockMatcher.compute_device call (Python checks + ctypes + the C-ABI's launch
path): N calls issued back to back on a tiny frame, host time per call, and the C1 frame rate with
3 streams when the host issues the calls.  usage: python tools/host_call_probe.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    res = {}
    for (H, W, D, name) in ((32, 128, 64, "tiny"), (480, 640, 64, "c1")):
        L, R, _ = stereo_pair(H, W, 0, D, seed=5)
        l, r = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
        m = HipBlockMatcher(device=0, num_disp=D, block_size=5)
        of = torch.empty((H, W), dtype=torch.int16, device=dev)
        ff = torch.empty((H, W), dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream(dev)
        for _ in range(50):
            m.compute_device(l, r, out_fixed=of, out_float=ff, stream=st)
        torch.cuda.synchronize()
        n = 2000
        t0 = time.perf_counter()
        for _ in range(n):
            m.compute_device(l, r, out_fixed=of, out_float=ff, stream=st)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res[name] = {"host_us_per_call": round((t1 - t0) / n * 1e6, 2), "total_us_per_call": round((t2 - t0) / n * 1e6, 2)}
        # the ctypes call alone (checks skipped): the C-ABI's own host cost
        from depthestimation_amd import _dsx
        lib, h = _dsx.lib(), m._handle()
        args = (h, l.data_ptr(), r.data_ptr(), H, W, W, of.data_ptr(), ff.data_ptr(), st.cuda_stream)
        t0 = time.perf_counter()
        for _ in range(n):
            lib.dsx_compute_device(*args)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        res[name]["cabi_only_host_us_per_call"] = round((t1 - t0) / n * 1e6, 2)
        m.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
