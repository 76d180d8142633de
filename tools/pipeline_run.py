"""The end_to_end leg's workload alone (bench.py pipeline_leg: 4 batches x 64 cfg2 queries from CHW
hypercolumns through fmpnp.pipeline.RefinePipeline), PASSES passes after one sizing pass -- for
rocprofv3 counter passes (tools/gpu_profile_pipeline.sh).  Prints the queries processed.
WINDOW=r (environment): windowed f-only packs of radius r (the bench's default), WINDOW=0 the full pack."""
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
nb, qb = 4, 64
batches, img = synth.pipeline_queries(nb, qb, 512, 256, 240, 320, device=dev, seed0=5000)
WINDOW = int(os.environ.get("WINDOW", "0")) or None
pipe = RefinePipeline(img, storage=torch.float32, depth=2, window=WINDOW,
                      model_kwargs=dict(n_iters=50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                        ratio_threshold=None))
for _ in range(1 + PASSES):
    pipe.run(batches)
torch.cuda.synchronize()
print(f"queries {(1 + PASSES) * nb * qb} window {WINDOW} refills {pipe.refills}")
