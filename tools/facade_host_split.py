"""Where the consumer call's time goes on the host (bench.py facade leg, one query per call):
wall time per feature_pnp call, the time inside fmpnp_feature_pnp (plan, uploads, launches and the
one stream wait), and the Python around it.  Compare with the call's kernel sum
(profiles/r05_pmc_facade_*.json kernel_us_per_call).

python tools/facade_host_split.py [SHAPE ...] [--calls N]
"""
import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]


def main():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="*", default=list(bench.FACADE_SHAPES))
    ap.add_argument("--calls", type=int, default=48)
    ap.add_argument("--profile", action="store_true", help="cProfile the calls (cumulative time per callee)")
    a = ap.parse_args()
    import torch
    from fmpnp import _lib, synth
    L = _lib.load()
    inner = L.fmpnp_feature_pnp
    spent = []

    class Timed:  # (ctypes function objects cannot be wrapped in place: the library handle's attribute is swapped)
        argtypes, restype = inner.argtypes, inner.restype

        def __call__(self, *args):
            t0 = time.perf_counter()
            rc = inner(*args)
            spent.append(time.perf_counter() - t0)
            return rc
    L.fmpnp_feature_pnp = Timed()
    dev = torch.device("cuda", 0)
    for name in a.shapes:
        spent.clear()
        if a.profile:
            import cProfile
            import pstats
            qs = bench.facade_queries(dev, synth, name)
            bench.facade_calls(dev, synth, name, calls=4, queries=qs)
            pr = cProfile.Profile()
            pr.enable()
            bench.facade_calls(dev, synth, name, calls=a.calls, warmup=0, queries=qs)
            pr.disable()
            print(f"== {name}: {a.calls} calls")
            pstats.Stats(pr).sort_stats("tottime").print_stats(30)
            continue
        d = bench.facade_calls(dev, synth, name, calls=a.calls)
        n = len(spent)
        c_ms = sorted(spent)[n // 2] * 1e3 if n else None
        print(json.dumps({"shape": name, "wall_ms_per_call": d["ms_per_call"], "c_call_ms_median": round(c_ms, 4),
                          "c_calls": n, "python_ms_per_call": round(d["ms_per_call"] - c_ms, 4)}), flush=True)
    L.fmpnp_feature_pnp = inner


if __name__ == "__main__":
    main()
