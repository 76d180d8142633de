"""f-only pack (FMPNP_LAYOUT_F channels-last copy) microbench over rotating distinct maps.

python tools/bench_pack_f.py [C H W ...]   prints us and GB/s (8C bytes per texel) per shape.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402

from fmpnp import _lib, synth  # noqa: E402

shapes = [(256, 240, 320), (512, 480, 640), (128, 480, 640), (512, 120, 160)]
if len(sys.argv) > 3:
    a = list(map(int, sys.argv[1:]))
    shapes = [tuple(a[i:i + 3]) for i in range(0, len(a), 3)]
dev = torch.device("cuda", 0)
L = _lib.load()
st = _lib.stream_ptr(dev)
for C, H, W in shapes:
    per = 8 * C * H * W
    NP = max(2, min(8, int(1.2e9 // per) + 1))
    fms = [synth.feature_map(C, H, W, 5 + i, dev) for i in range(NP)]
    outs = [torch.empty((H, W, C), dtype=torch.float32, device=dev) for _ in range(NP)]

    def pack(i):
        _lib.check(L.fmpnp_pack_features_f(ctypes.c_void_p(fms[i % NP].data_ptr()), _lib.F32, C, H, W,
                                           ctypes.c_void_p(outs[i % NP].data_ptr()), _lib.F32, C, st), "pack_f")
    for i in range(NP):
        pack(i)
    torch.cuda.synchronize()
    reps = 10 * NP
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(reps):
        pack(i)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    print(f"pack_f C={C} {H}x{W}: {ms * 1e3:.1f} us  {per / (ms / 1e3) / 1e9:.0f} GB/s  (CT={os.environ.get('FMPNP_PACK_F_CT', '64')} XT={os.environ.get('FMPNP_PACK_F_XT', '32')})",
          flush=True)
    del fms, outs
