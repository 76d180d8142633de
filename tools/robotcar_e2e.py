"""bench.py's robotcar_1664 end-to-end workload (2 x 32 queries, C = 1664 at 256x256, N = 866, the
channel levels of default_robotcar.gin:75 through RefinePipeline) for several workgroups-per-query
settings of the LM launches (0: the planner's choice, auto: the pipeline's default).
Usage: python tools/robotcar_e2e.py [wgs|auto ...]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import numpy as np
import torch
import fmpnp
from fmpnp import _lib, synth
from fmpnp.pipeline import RefinePipeline

WGS = [None if w == "auto" else int(w) for w in sys.argv[1:]] or [1, None]
dev = torch.device("cuda", 0)
batches, img = synth.pipeline_queries(2, 32, 866, 1664, 256, 256, device=dev, seed0=7000)
ref = None
for w in WGS:
    pipe = RefinePipeline(img, storage=torch.float32, depth=2, wgs_per_problem=w,
                          levels=[(640, 1664), (128, 640), (0, 128)],
                          model_kwargs=dict(n_iters=50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                            ratio_threshold=None))
    out = pipe.run(batches)
    g = _lib.last_launch()["wgs_per_problem"]
    if ref is None:
        ref = out
    same = all(np.array_equal(a["R"], b["R"]) and np.array_equal(a["t"], b["t"]) for x, y in zip(ref, out)
               for a, b in zip(x, y))
    best = None
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipe.run(batches)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    print(f"wgs {w} (G {g}): {64 / best:8.1f} queries/s  identical {same}", flush=True)
