"""Per-evaluation durations of the LM kernel (FMPNP_DBG=4: s_memtime at the start of each
evaluation of every team's first problem).  Usage: FMPNP_DBG=4 python tools/diag_evals.py [B] [G] [init]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import numpy as np, torch
from fmpnp import _lib, refine as rf, synth

assert int(os.environ.get("FMPNP_DBG", "0")) & 4, "run with FMPNP_DBG=4"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
wgs = int(sys.argv[2]) if len(sys.argv) > 2 else 0
init = sys.argv[3] if len(sys.argv) > 3 else "easy"
dev = torch.device("cuda", 0)
probs = []
for q in range(B):
    inp = synth.problem_inputs(512, 256, 240, 320, seed=q, device=dev, init=init)
    feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev)
    probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                 inp["R0"], inp["t0"]))
opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=wgs)
ab = rf.AsyncBatch(probs, opts)
for _ in range(3):
    ab.launch()
torch.cuda.synchronize()
L = _lib.load()
L.fmpnp_debug_stamps.argtypes = [ctypes.c_void_p]
info = _lib.last_launch()
st = torch.zeros(info["grid"] * 64, dtype=torch.int64, device=dev)
L.fmpnp_debug_stamps(ctypes.c_void_p(st.data_ptr()))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); ab.launch(); e1.record(); torch.cuda.synchronize()
L.fmpnp_debug_stamps(None)
res = ab.results()
ne = int(np.median([r["n_evals"] for r in res]))
t = st.view(-1, 64).cpu().numpy().astype(np.float64)
t = t[t[:, 0] > 0]
d = np.diff(t[:, :ne + 1], axis=1)  # [wg][eval] cycles
m = d.mean(0)
print(f"B={B} launch={info} stamped launch {e0.elapsed_time(e1):.3f} ms; {len(t)} workgroups, {ne} evals")
print(f"total cycles per problem (mean over WGs): {d.sum(1).mean():.0f}; eval0 {m[0]:.0f}; evals 1.. mean {m[1:].mean():.0f}"
      f" median {np.median(m[1:]):.0f}")
print("per-eval mean cycles:", " ".join(f"{x:.0f}" for x in m))
print("per-eval max  cycles:", " ".join(f"{x:.0f}" for x in d.max(0)))
