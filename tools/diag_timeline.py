"""Timeline of one LM evaluation across the 8 waves of each workgroup (FMPNP_DBG bit 4: absolute
s_memtime at the tl_stamp sites of evaluation E of every team's first problem), cycles relative
to the evaluation's start, mean over workgroups.
Usage: python tools/diag_timeline.py [B] [E] [init]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
E = int(sys.argv[2]) if len(sys.argv) > 2 else 20
init = sys.argv[3] if len(sys.argv) > 3 else "easy"
os.environ["FMPNP_DBG"] = str(16 | (E << 8))
import numpy as np, torch
from fmpnp import _lib, refine as rf, synth

SITES = ["start", "projected", "gathered", "contrib", "pre-barrier", "barrier1", "combined", "bookkeeping",
         "solved", "pose stored", "spec done", "barrier2", "acc operands", "acc ldlt", "acc decided", "ratio checked"]
dev = torch.device("cuda", 0)
probs = []
for q in range(B):
    inp = synth.problem_inputs(512, 256, 240, 320, seed=q, device=dev, init=init)
    feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev)
    probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                 inp["R0"], inp["t0"]))
ratio = float(os.environ["RATIO"]) if os.environ.get("RATIO") else None  # ratio test (model.py:324-336)
opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, ratio_threshold=ratio, dtype=_lib.F32)
ab = rf.AsyncBatch(probs, opts)
for _ in range(3):
    ab.launch()
torch.cuda.synchronize()
L = _lib.load()
L.fmpnp_debug_stamps.argtypes = [ctypes.c_void_p]
info = _lib.last_launch()
st = torch.zeros(info["grid"] * 8 * 16, dtype=torch.int64, device=dev)
L.fmpnp_debug_stamps(ctypes.c_void_p(st.data_ptr()))
ab.launch()
torch.cuda.synchronize()
L.fmpnp_debug_stamps(None)
t = st.view(-1, 8, 16).cpu().numpy().astype(np.float64)
t = t[t[:, 0, 0] > 0]
rel = t - t[:, 0:1, 0:1]
rel[t == 0] = np.nan
m = np.nanmean(rel, 0)
print(f"B={B} eval {E} ({init}), {len(t)} workgroups, cycles since wave 0's start (mean over WGs)")
print("site".ljust(13) + "".join(f"   w{w:d}  " for w in range(8)))
for k, name in enumerate(SITES):
    if np.all(np.isnan(m[:, k])):
        continue
    print(name.ljust(13) + "".join("   ----  " if np.isnan(m[w, k]) else f"{m[w, k]:7.0f}  " for w in range(8)))
med = np.nanmedian(rel, 0)
print("median over workgroups (wave 0):", "  ".join(f"{SITES[k]} {med[0, k]:.0f}" for k in range(len(SITES))
                                                      if not np.isnan(med[0, k])))
# the slowest wave of each workgroup sets its barrier: mean over workgroups of the per-WG maximum
for k in (3, 4, 10):
    v = rel[:, :, k]
    if np.all(np.isnan(v)):
        continue
    print(f"{SITES[k]:13s} per-WG max over waves: mean {np.nanmean(np.nanmax(v, 1)):7.0f}; "
          f"argmax wave histogram {np.bincount(np.nanargmax(np.where(np.isnan(v), -1e18, v), 1), minlength=8).tolist()}")
