"""Workgroups per problem (G) on the RobotCar production pyramid (bench.py pyramid_leg's workload:
C = 1664 at 256x256, N points (environment N, default 866; 295 the median query), B queries, the
default_robotcar.gin:75 channel levels): ms per level launch for each G (0: the planner's choice).
Usage: [N=295] python tools/pyramid_g_sweep.py [B] [G ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402

from fmpnp import _lib, refine as rf, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
GS = [int(x) for x in sys.argv[2:]] or [0, 1, 2, 4, 8]
dev = torch.device("cuda", 0)
levels = [(640, 1664), (128, 640), (0, 128)]
feats, frefs, inps = [], [], []
for q in range(B):
    inp = synth.problem_inputs(int(os.environ.get("N", "866")), 1664, 256, 256, seed=20000 + q, device=dev,
                               init="easy")
    feats.append(rf.pack_features(inp.pop("fmap"), storage=torch.float32, device=dev))
    frefs.append(inp.pop("fref"))
    inps.append(inp)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for G in GS:
    opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=G)
    R = [i["R0"] for i in inps]
    t = [i["t0"] for i in inps]
    row = []
    for cb, ce in levels:
        ps = [rf.make_problem(feats[q], frefs[q], inps[q]["pts3d"], inps[q]["K"], inps[q]["im_width"],
                              inps[q]["im_height"], R[q], t[q], c_begin=cb, c_end=ce) for q in range(B)]
        ab = rf.AsyncBatch(ps, opts)
        for _ in range(3):
            ab.launch()
        torch.cuda.synchronize()
        s.record()
        for _ in range(10):
            ab.launch()
        e.record()
        torch.cuda.synchronize()
        res = ab.results()
        row.append((cb, ce, s.elapsed_time(e) / 10, _lib.last_launch()["wgs_per_problem"]))
        R = [r["R"] for r in res]
        t = [r["t"] for r in res]
    print(f"G={G}: " + "  ".join(f"[{cb}:{ce}] {ms:.4f} ms (G {g})" for cb, ce, ms, g in row) +
          f"  total {sum(r[2] for r in row):.4f} ms", flush=True)
