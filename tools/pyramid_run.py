"""bench.py's pyramid_robotcar_1664 workload alone, for rocprofv3 counter passes
(tools/gpu_profile_pyramid.sh): B=32 queries of C=1664 256x256 hypercolumns, N points, the three
channel levels of input_configs/default_robotcar.gin:75, each level's launch REPS times in a row
(level 0 first).  usage: python tools/pyramid_run.py N [REPS]"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402
from fmpnp import _lib, refine as rf, synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 866
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 4
LEVELS = [(640, 1664), (128, 640), (0, 128)]
dev = torch.device("cuda", 0)
feats, frefs, inps = [], [], []
for q in range(32):
    inp = synth.problem_inputs(N, 1664, 256, 256, seed=20000 + q, device=dev, init="easy")
    feats.append(rf.pack_features(inp.pop("fmap"), storage=torch.float32, device=dev))
    frefs.append(inp.pop("fref"))
    inps.append(inp)
opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
R = [i["R0"] for i in inps]
t = [i["t0"] for i in inps]
for cb, ce in LEVELS:
    ps = [rf.make_problem(feats[q], frefs[q], inps[q]["pts3d"], inps[q]["K"], inps[q]["im_width"],
                          inps[q]["im_height"], R[q], t[q], c_begin=cb, c_end=ce) for q in range(32)]
    ab = rf.AsyncBatch(ps, opts)
    for _ in range(REPS):
        ab.launch()
    res = ab.results()
    R = [r["R"] for r in res]
    t = [r["t"] for r in res]
torch.cuda.synchronize()
print(f"levels {len(LEVELS)} reps {REPS}")
