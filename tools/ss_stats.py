"""Steady-state gather helpers (VAR_GM_SS): per evaluation, how many dirty points the helper's
records served and how many the main still gathered on demand, by FMPNP_SS_CAP (FMPNP_DBG bit 6
counts the served ones in texel_gathers' high word).  B=128 cfg2 queries, the bench's seeds.
The helpers are opt-in: FMPNP_SS=1 (records handed over, default here) or SS_MODE=2 (prefetch only).
Usage: [SS_MODE=1|2] python tools/ss_stats.py [init] [caps...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch
from fmpnp import _lib, refine as rf, synth

init = sys.argv[1] if len(sys.argv) > 1 else "easy"
caps = [int(c) for c in sys.argv[2:]] or [1, 2, 4, 8, 16]
dev = torch.device("cuda", 0)
probs = []
for q in range(128):
    inp = synth.problem_inputs(512, 256, 240, 320, seed=q, device=dev, init=init)
    f = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev)
    probs.append(rf.make_problem(f, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                 inp["R0"], inp["t0"]))
opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
os.environ["FMPNP_SS"] = "0"
base = rf.AsyncBatch(probs, opts)
base.launch()
r0 = base.results()
g0 = sum(r["texel_gathers"] for r in r0)
ev = sum(r["n_evals"] for r in r0)
t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t[0].record()
for _ in range(20):
    base.launch()
t[1].record()
torch.cuda.synchronize()
print(f"{init}: spec only: gathers {g0} ({g0 / ev:.2f} per problem-evaluation, first evaluations included), "
      f"{t[0].elapsed_time(t[1]) / 20:.4f} ms per launch")
os.environ["FMPNP_SS"] = os.environ.get("SS_MODE", "1")
os.environ["FMPNP_DBG"] = "64"
for cap in caps:
    os.environ["FMPNP_SS_CAP"] = str(cap)
    ab = rf.AsyncBatch(probs, opts)
    ab.launch()
    rs = ab.results()
    served = sum(r["texel_gathers"] >> 32 for r in rs)
    tot = sum(r["texel_gathers"] & 0xFFFFFFFF for r in rs)
    t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t[0].record()
    for _ in range(20):
        ab.launch()
    t[1].record()
    torch.cuda.synchronize()
    print(f"cap {cap:2d}: served {served} ({served / ev:.2f}/eval), main gathers {tot - served} "
          f"({(tot - served) / ev:.2f}/eval), {t[0].elapsed_time(t[1]) / 20:.4f} ms per launch", flush=True)
