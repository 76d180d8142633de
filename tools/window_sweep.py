"""End-to-end pipeline (bench.py end_to_end: 4 batches x 64 cfg2 queries from CHW maps) with the
full f-only pack and with windowed packs of several radii: queries/s and refills per run.
Usage: python tools/window_sweep.py [init] [radii...]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import numpy as np
import torch
import fmpnp
from fmpnp import synth
from fmpnp.pipeline import RefinePipeline

init = sys.argv[1] if len(sys.argv) > 1 else "easy"
radii = [None] + [int(r) for r in sys.argv[2:]] if len(sys.argv) > 2 else [None, 4, 5, 6, 8]
dev = torch.device("cuda", 0)
batches, img = synth.pipeline_queries(4, 64, 512, 256, 240, 320, device=dev, seed0=5000)
if init != "easy":
    R0, t0 = synth.INITS[init]
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R0, t0
    batches = [[(a, b, p._replace(matrix=T), k) for (a, b, p, k) in qs] for qs in batches]
ref = None
for r in radii:
    pipe = RefinePipeline(img, storage=torch.float32, depth=2, window=r,
                          model_kwargs=dict(n_iters=50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                            ratio_threshold=None))
    out = pipe.run(batches)
    if ref is None:
        ref = out
    same = all(np.array_equal(a["R"], b["R"]) and np.array_equal(a["t"], b["t"]) for x, y in zip(ref, out)
               for a, b in zip(x, y))
    best = None
    for _ in range(3):
        pipe.refills = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipe.run(batches)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    print(f"{init} window {r}: {256 / best:9.1f} queries/s  refills/run {pipe.refills}  identical {same}", flush=True)
