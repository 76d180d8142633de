"""Does an async H2D upload from pinned memory block the host while its stream is busy?
A ~2 ms sleep kernel is queued on a side stream, then the upload's host time is measured
(torch .to(non_blocking=True) from a pinned tensor, and copy_ into a preallocated device tensor).

python tools/h2d_block_probe.py
"""
import time

import torch

dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
n = 64 * 2560  # one pipeline batch's points and inliers (fp64)
pinned = torch.empty(n, dtype=torch.float64, pin_memory=True)
dst = torch.empty(n, dtype=torch.float64, device=dev)
torch.cuda._sleep(1000)
torch.cuda.synchronize()
cyc = int(2e-3 * 2.1e9)  # about 2 ms of device sleep
for name in ("to", "copy_", "idle_to"):
    for rep in range(3):
        with torch.cuda.stream(s):
            if name != "idle_to":
                torch.cuda._sleep(cyc)
            t0 = time.perf_counter()
            if name == "copy_":
                dst.copy_(pinned, non_blocking=True)
            else:
                pinned.to(dev, non_blocking=True)
            t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name:8s} host {1e3 * (t1 - t0):7.3f} ms  (until idle {1e3 * (t2 - t0):7.3f} ms)", flush=True)
