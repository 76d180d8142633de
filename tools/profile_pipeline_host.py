"""Host-side profile of fmpnp.pipeline.RefinePipeline.run (cProfile, top functions by
own time) -- where the per-query Python overhead of the end-to-end path goes.

python tools/profile_pipeline_host.py [n_batches] [batch]
"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402

import fmpnp  # noqa: E402
from fmpnp import synth  # noqa: E402
from fmpnp.pipeline import RefinePipeline  # noqa: E402

NB = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda", 0)
batches, img = synth.pipeline_queries(NB, B, device=dev)
pipe = RefinePipeline(img, storage=torch.float32, depth=2, window=int(os.environ.get("WINDOW", "0")) or None,
                      model_kwargs=dict(n_iters=50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                        ratio_threshold=None))
pipe.run(batches)
torch.cuda.synchronize()
pr = cProfile.Profile()
if os.environ.get("PREP_ONLY"):  # one batch's host preparation, 10 times (cumulative time per callee)
    import time
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(10):
        pipe._prepare(list(batches[0]), 0)
    pr.disable()
    torch.cuda.synchronize()
    print(f"_prepare: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per batch of {B} (profiled)")
    pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
    sys.exit(0)
pr.enable()
pipe.run(batches)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
