"""ms per LM launch with and without the speculative next-texel gathers, over batch sizes
(cfg2 shape, GM, 50 iterations, fp32 packed layout): the planner's speculation rule."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import numpy as np, torch
from fmpnp import _lib, refine as rf, synth

dev = torch.device("cuda", 0)
Bs = [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "1,16,64,128,192,256,512").split(",")]
init = os.environ.get("INIT", "easy")
probs = []
for q in range(max(Bs)):
    inp = synth.problem_inputs(512, 256, 240, 320, seed=q, device=dev, init=init)
    f = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev)
    probs.append(rf.make_problem(f, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                 inp["R0"], inp["t0"]))
    del inp
for B in Bs:
    row = []
    for spec in (True, False):
        ab = rf.AsyncBatch(probs[:B], rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, speculate=spec))
        ab.launch(); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        s.record()
        for _ in range(reps):
            ab.launch()
        e.record(); torch.cuda.synchronize()
        row.append(s.elapsed_time(e) / reps)
    print(f"B={B:5d} spec {row[0]:.4f} ms  no-spec {row[1]:.4f} ms  ratio {row[0] / row[1]:.3f}", flush=True)
