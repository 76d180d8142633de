"""Where an LM launch's time goes at any shape (a stamps build: tools/build_ab.sh stamps -- -DFMPNP_STAMPS=1,
run with FMPNP_LIB_PATH=ab_old/stamps/libfmpnp.so): per-wave phase cycles (fmpnp_debug_stamps) and the
per-evaluation durations (FMPNP_DBG=4) of the team's first problem.

  python tools/diag_level.py N C H W c_begin c_end B [wgs]     e.g. 295 1664 256 256 640 1664 1
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmpnp import _lib, refine as rf, synth  # noqa: E402

N, C, H, W, cb, ce, B = (int(x) for x in sys.argv[1:8])
wgs = int(sys.argv[8]) if len(sys.argv) > 8 else 0
dev = torch.device("cuda", 0)
probs = []
for q in range(B):
    inp = synth.problem_inputs(N, C, H, W, seed=20000 + q, device=dev)
    feats = rf.pack_features(inp.pop("fmap"), storage=torch.float32, device=dev)
    probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                 inp["R0"], inp["t0"], c_begin=cb, c_end=ce))
opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=wgs)
ab = rf.AsyncBatch(probs, opts)
for _ in range(3):
    ab.launch()
torch.cuda.synchronize()
info = _lib.last_launch()
L = _lib.load()
L.fmpnp_debug_stamps.argtypes = [ctypes.c_void_p]
plain = []
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ab.launch()
    e1.record()
    torch.cuda.synchronize()
    plain.append(e0.elapsed_time(e1))
res = ab.results()
evals = float(np.mean([r["n_evals"] for r in res]))
gath = sum(r["texel_gathers"] for r in res)
print(f"N={N} C={ce - cb} (of {C}) {H}x{W} B={B} launch={info}")
print(f"plain launch median {np.median(plain):.4f} ms; {evals:.1f} evals/problem; texel gathers "
      f"{gath / max(1, B * evals * N) * 100:.1f} % of point-evaluations")
# phase cycles per wave (FMPNP_DBG unset)
os.environ.pop("FMPNP_DBG", None)
st = torch.zeros(info["grid"] * 8 * 13, dtype=torch.int64, device=dev)
L.fmpnp_debug_stamps(ctypes.c_void_p(st.data_ptr()))
ab.launch()
torch.cuda.synchronize()
L.fmpnp_debug_stamps(None)
phw = st.view(-1, 8, 13).cpu().numpy().astype(np.float64)[:info["grid"] if info["helpers"] == 0 else B]
names = ["proj", "gather", "loss+contrib", "wait/exch", "combine|spec", "LM state", "solve", "pose+sync",
         "e0 proj", "e0 gather", "e0 l+c", "e0 wait", "w0 spec"]
print("cycles per steady-state evaluation, mean over workgroups (phases 0-7), first evaluation (8-11):")
for w in range(8):
    u = phw[:, w, :].mean(0)
    print(f"  wave {w}: " + " ".join(f"{names[k]} {u[k] / (max(evals - 1, 1) if k < 8 else 1):7.0f}" for k in range(13)))
# per-evaluation durations (FMPNP_DBG=4)
os.environ["FMPNP_DBG"] = "4"
st2 = torch.zeros(info["grid"] * 64, dtype=torch.int64, device=dev)
L.fmpnp_debug_stamps(ctypes.c_void_p(st2.data_ptr()))
ab.launch()
torch.cuda.synchronize()
L.fmpnp_debug_stamps(None)
os.environ.pop("FMPNP_DBG")
ne = int(np.median([r["n_evals"] for r in res]))
t = st2.view(-1, 64).cpu().numpy().astype(np.float64)
t = t[t[:, 0] > 0]
d = np.diff(t[:, :ne + 1], axis=1)
m = d.mean(0)
print(f"cycles per problem {d.sum(1).mean():.0f}: eval0 {m[0]:.0f}, evals 1.. mean {m[1:].mean():.0f} "
      f"median {np.median(m[1:]):.0f}")
print("per-eval mean cycles:", " ".join(f"{x:.0f}" for x in m))
