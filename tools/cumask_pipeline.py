"""CU-masked streams for the end-to-end pipeline (experiment): the f-only pack of 128 cfg2 maps on a
stream restricted to a subset of the CUs (hipExtStreamCreateWithCUMask), alone and beside the LM
launch of another 128 queries on a stream restricted to the complementary CUs.
Usage: python tools/cumask_pipeline.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402

from fmpnp import _lib, refine as rf, synth  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
hip = ctypes.CDLL("libamdhip64.so")
ncu = torch.cuda.get_device_properties(dev).multi_processor_count
B, C, H, W = 128, 256, 240, 320


def masked_stream(bits):
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


maps = [synth.feature_map(C, H, W, 900 + i, dev) for i in range(B)]
outs = [torch.empty((H, W, C), dtype=torch.float32, device=dev) for _ in range(B)]
L = _lib.load()
vp = ctypes.c_void_p
shape = (ctypes.c_int * (4 * B))(*([C, H, W, C] * B))


def pack(stream):
    with torch.cuda.stream(stream):
        rc = L.fmpnp_pack_features_batch(B, (vp * B)(*[m.data_ptr() for m in maps]),
                                         (vp * B)(*[o.data_ptr() for o in outs]), shape, _lib.F32, _lib.F32,
                                         0, 0, _lib.LAYOUT_F, _lib.stream_ptr(dev))
        _lib.check(rc, "pack")


probs = []
for q in range(B):
    inp = synth.problem_inputs(512, C, H, W, seed=q, device=dev)
    f = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev, layout="f")
    probs.append((f, rf.make_problem(f, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                     inp["R0"], inp["t0"])))
opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=1, helpers=-1)
opts.layout = _lib.LAYOUT_F
ab = rf.AsyncBatch([p for _, p in probs], opts)


def lm(stream):
    with torch.cuda.stream(stream):
        ab.launch(_lib.stream_ptr(dev))


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


full = torch.cuda.Stream(dev)
half_hi = masked_stream(range(ncu // 2, ncu))
half_lo = masked_stream(range(0, ncu // 2))
odd = masked_stream(range(1, ncu, 2))
even = masked_stream(range(0, ncu, 2))
print(f"CUs {ncu}", flush=True)
print(f"pack 128 maps, all CUs:        {timed(lambda: pack(full)):.3f} ms", flush=True)
print(f"pack 128 maps, CUs {ncu // 2}-{ncu - 1}:    {timed(lambda: pack(half_hi)):.3f} ms", flush=True)
print(f"pack 128 maps, odd CUs:        {timed(lambda: pack(odd)):.3f} ms", flush=True)
print(f"LM 128 queries, all CUs:       {timed(lambda: lm(full)):.3f} ms", flush=True)
print(f"LM 128 queries, CUs 0-{ncu // 2 - 1}:     {timed(lambda: lm(half_lo)):.3f} ms", flush=True)
print(f"LM 128 queries, even CUs:      {timed(lambda: lm(even)):.3f} ms", flush=True)


def both(ps, ls):
    def f():
        pack(ps)
        lm(ls)
    return f


print(f"pack || LM, unmasked streams:  {timed(both(full, torch.cuda.Stream(dev))):.3f} ms", flush=True)
print(f"pack hi || LM lo:              {timed(both(half_hi, half_lo)):.3f} ms", flush=True)
print(f"pack odd || LM even:           {timed(both(odd, even)):.3f} ms", flush=True)
