"""PCIe copy rates on the GPU box (context for bench.py's e2e_host): pinned H2D, D2H, both at once
on two streams, for a C2 frame pair (4.1 MB up) and its int16 map (4.1 MB down).  Dev tool."""
import json
import time

import torch

dev = torch.device("cuda:0")
n = 1920 * 1080 * 2
h_in = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h_out = torch.empty(n, dtype=torch.uint8, pin_memory=True)
d_in = torch.empty(n, dtype=torch.uint8, device=dev)
d_out = torch.empty(n, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
res = {}


def run(name, fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t) / reps
    res[name] = {"us_per_rep": round(dt * 1e6, 1), "GB_s_per_direction": round(n / dt / 1e9, 1)}


def h2d():
    with torch.cuda.stream(s1):
        d_in.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_out, non_blocking=True)


def both():
    h2d()
    d2h()


def both_same_stream():
    with torch.cuda.stream(s1):
        d_in.copy_(h_in, non_blocking=True)
        h_out.copy_(d_out, non_blocking=True)


run("h2d_4MB", h2d)
run("d2h_4MB", d2h)
run("h2d_and_d2h_two_streams", both)
run("h2d_then_d2h_one_stream", both_same_stream)
print(json.dumps({"bytes_per_copy": n, "results": res}))
