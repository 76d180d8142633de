"""End-to-end pipeline throughput vs the LM launch's workgroups per query (0 = planner,
1 = one workgroup per query) and the batch size.  python tools/pipe_ab.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402

import fmpnp  # noqa: E402
from fmpnp import _lib, synth  # noqa: E402
from fmpnp.pipeline import RefinePipeline  # noqa: E402

dev = torch.device("cuda", 0)
kw = dict(n_iters=50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01, ratio_threshold=None)
for nb, qb in ((4, 64), (4, 128), (8, 32)):
    batches, img = synth.pipeline_queries(nb, qb, device=dev, seed0=5000)
    for wgs in (0, 1):
        pipe = RefinePipeline(img, storage=torch.float32, depth=2, model_kwargs=kw, wgs_per_problem=wgs)
        ref = pipe.run(batches)
        best = None
        for _ in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            out = pipe.run(batches)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        print(f"batches {nb} x {qb}  wgs {wgs}: {nb * qb / best:9.1f} queries/s  launch {_lib.last_launch()}", flush=True)
    del batches
    torch.cuda.empty_cache()
