"""The end_to_end leg's workload alone (bench.py pipeline_leg: 4 batches x 64 cfg2 queries from CHW
hypercolumns through fmpnp.pipeline.RefinePipeline), PASSES passes after one sizing pass -- for
rocprofv3 counter passes (tools/gpu_profile_pipeline.sh).  Prints the queries processed.
WINDOW=r (environment): windowed f-only packs of radius r (the bench's default), WINDOW=0 the full pack.
ROBOTCAR=1: bench.py's robotcar_1664 workload instead (2 x 32 queries, C = 1664 at 256x256, N = 866,
the three channel levels of default_robotcar.gin:75)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402
import fmpnp  # noqa: E402
from fmpnp import synth  # noqa: E402
from fmpnp.pipeline import RefinePipeline  # noqa: E402

PASSES = int(sys.argv[1]) if len(sys.argv) > 1 else 2
dev = torch.device("cuda", 0)
ROBOTCAR = os.environ.get("ROBOTCAR") == "1"
if ROBOTCAR:
    nb, qb = 2, 32
    batches, img = synth.pipeline_queries(nb, qb, 866, 1664, 256, 256, device=dev, seed0=7000)
else:
    nb, qb = 4, 64
    batches, img = synth.pipeline_queries(nb, qb, 512, 256, 240, 320, device=dev, seed0=5000)
WINDOW = int(os.environ.get("WINDOW", "0")) or None
pipe = RefinePipeline(img, storage=torch.float32, depth=2, window=WINDOW,
                      levels=[(640, 1664), (128, 640), (0, 128)] if ROBOTCAR else None,
                      model_kwargs=dict(n_iters=50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                        ratio_threshold=None))
for _ in range(1 + PASSES):
    pipe.run(batches)
torch.cuda.synchronize()
print(f"queries {(1 + PASSES) * nb * qb} window {WINDOW} refills {pipe.refills}")
