"""Phase shares of the LM kernel from the debug s_memtime stamps (fmpnp_debug_stamps)."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import numpy as np, torch
from fmpnp import _lib, refine as rf, synth

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
wgs = int(sys.argv[2]) if len(sys.argv) > 2 else 0
layout = sys.argv[3] if len(sys.argv) > 3 else "fgrad"   # "f": FMPNP_LAYOUT_F
dev = torch.device("cuda", 0)
probs = []
for q in range(B):
    inp = synth.problem_inputs(512, 256, 240, 320, seed=q, device=dev)
    feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev, layout=layout)
    probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"], inp["R0"], inp["t0"]))
spec = os.environ.get("SPEC", "1") == "1"
sampling = os.environ.get("SAMPLING", "nearest")  # bilinear: phases 0/1/2 = project / memo build / sums+loss+contrib
opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=wgs, speculate=spec,
                       sampling=sampling, memoize=os.environ.get("MEMO", "1") == "1")
ab = rf.AsyncBatch(probs, opts)
ab.launch(); torch.cuda.synchronize()
L = _lib.load()
L.fmpnp_debug_stamps.argtypes = [ctypes.c_void_p]
info = _lib.last_launch()
st = torch.zeros(info["grid"] * 8 * 13, dtype=torch.int64, device=dev)
L.fmpnp_debug_stamps(ctypes.c_void_p(st.data_ptr()))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); ab.launch(); e1.record(); torch.cuda.synchronize()
L.fmpnp_debug_stamps(None)
plain = []
for _ in range(10):
    e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e2.record(); ab.launch(); e3.record(); torch.cuda.synchronize()
    plain.append(e2.elapsed_time(e3))
phw = st.view(-1, 8, 13).cpu().numpy().astype(np.float64)
ph = phw[:, 0, :]
res = ab.results()
g = sum(r["texel_gathers"] for r in res)
full = sum(r["n_evals"] for r in res) * 512
print(f"texel gathers {g} of {full} point-evals ({100.0 * g / max(full, 1):.1f} %)")
names = ["proj (w0)", "gather (w0)", "loss+contrib", "wait/exchange", "combine", "LM state", "solve",
         "pose+sync", "eval0 proj", "eval0 gather", "eval0 l+c", "eval0 wait", "w0 spec"]
tot = ph.sum(0)
print(f"B={B} launch={info} stamped launch {e0.elapsed_time(e1):.3f} ms, plain launch median {np.median(plain):.3f} ms (min {min(plain):.3f}) -> {B / np.median(plain) * 1e3:.0f} /s")
for k in range(13):
    print(f"  {names[k]:12s} {100 * tot[k] / tot.sum():6.2f} %   mean per WG {ph[:, k].mean() / 1e3:10.1f} kcyc")
evals = sum(r["n_evals"] for r in res) / max(len(res), 1)
print(f"per-wave phases 0-2 (steady state, cycles per evaluation, mean over WGs; {evals:.0f} evals/problem):")
for w in range(8):
    v = phw[:, w, :3].mean(0) / max(evals - 1, 1)
    u = phw[:, w, :].mean(0) / max(evals - 1, 1)
    print(f"  wave {w}: proj {v[0]:7.0f}  gather {v[1]:7.0f}  loss+contrib {v[2]:7.0f}  sum {v.sum():7.0f}"
          f"  | spec(slot4/12) {u[4] if w else u[12]:7.0f}  after-barrier(slot7) {u[7]:7.0f}"
          + (f"  [barrier {u[3]:6.0f} census {u[5]:6.0f} issue {u[6]:6.0f}]" if w else ""))
