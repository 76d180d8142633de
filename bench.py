#!/usr/bin/env python3
"""Benchmark: feature-metric PnP refinements/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1] shape, batched as configs[2]): every GPU refines
its own batch of B independent queries, each N=512 points, C=256 channels,
240x320 hypercolumn (960x1280 image, stride 4), Geman-McClure, lambda0=0.01,
50 LM iterations, fp32 texels / fp64 arithmetic.  Synthetic inputs (SURVEY.md
§8d recipe; no dataset or CNN weights offline).  One step = one launch of the
LM kernel over the whole batch (all 50 iterations of all B queries), with the
packed features already resident in HBM.  Weak scaling: B queries per GPU;
at 8 GPUs and B=128 this is configs[2] (1024 queries).  No collectives on the
data path: ranks only meet in the timing barriers.

Also reported: single-query latency (B=1, one query spread over several
workgroups), the feature-pack kernel (fused Sobel + channels-last) rate, the
end-to-end rate from CHW hypercolumns (pack + reference gather + LM through
fmpnp.pipeline, wall clock), the roofline of the LM kernel, and the CPU baseline (the oracle's C restatement of
the reference loop, OpenMP over queries) on a bounded sample.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

N_PTS, C, HF, WF, ITERS = 512, 256, 240, 320, 50
HBM_PEAK = 8.0e12  # MI355X HBM3E spec (MI355X_MICROARCH.md)
B_ITER = N_PTS * (16 * C + 24)  # algorithmic bytes per GN iteration per query


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=128, help="queries per GPU")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="total queries split over the GPUs (strong scaling); 0 = --batch per GPU (weak)")
    ap.add_argument("--wgs", type=int, default=0, help="workgroups per query (0 = auto)")
    ap.add_argument("--cpu-sample", type=int, default=1024, help="queries in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-extras", action="store_true", help="skip single-query / pack / CPU legs")
    ap.add_argument("--no-nomemo", action="store_true", help="skip the memoisation-off comparison launch")
    ap.add_argument("--no-bilinear", action="store_true", help="skip the bilinear-sampling launch")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the end-to-end (pack + gather + LM) leg")
    ap.add_argument("--no-layout-f", action="store_true", help="skip the f-only layout launch")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # one process per GPU; FMPNP_BENCH_BACKEND=gloo (and more ranks than GPUs) rehearses the
    # distributed path on a one-GPU box -- the timing barrier and max-over-ranks only
    backend = os.environ.get("FMPNP_BENCH_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    gpu = local % ndev
    if dist:
        import torch.distributed as tdist
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            tdist.init_process_group(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    import fmpnp
    from fmpnp import _lib, refine as rf, synth

    # ---------------- setup (untimed): this rank's queries, packed in HBM ----------------
    # weak scaling (default): B queries per GPU; --global-batch G: G queries split over the
    # ranks (SURVEY.md 8e's fixed-total form, e.g. 1024), strong scaling
    B = -(-args.global_batch // world) if args.global_batch > 0 else args.batch
    t0 = time.time()
    probs = []
    keep = []
    for q in range(B):
        seed = rank * 100003 + q
        inp = synth.problem_inputs(N_PTS, C, HF, WF, seed=seed, device=dev)
        feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev)
        probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"],
                                     inp["im_height"], inp["R0"], inp["t0"]))
        if q < 1:
            keep.append(inp)
        del inp
    torch.cuda.synchronize()
    if rank == 0:
        log(f"[bench] setup {B} queries/GPU in {time.time() - t0:.1f}s "
            f"({torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB resident)")
    opts = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=args.wgs)
    batch = rf.AsyncBatch(probs, opts)

    # ---------------- warmup ----------------
    for _ in range(args.warmup):
        batch.launch()
    torch.cuda.synchronize()
    launch = _lib.last_launch()

    # ---------------- timed region ----------------
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        batch.launch()
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t_start
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    if dist:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = batch.results()
    statuses = sorted({r["status"] for r in res})
    if any(s & _lib.STATUS_SYNC_TIMEOUT for s in statuses):
        raise RuntimeError("sync timeout in the LM kernel")

    value = B * world * args.steps / elapsed
    ms_step = 1e3 * elapsed / args.steps
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    algo_bytes = B * ITERS * B_ITER
    achieved = algo_bytes / avg_kernel_s
    # bytes the memoised kernel actually gathers: 16C per point-texel gather (f, gx, gy, fref
    # fp32) + the fp64 points read once per query
    gathers = int(sum(r["texel_gathers"] for r in res))
    gathered_bytes = gathers * 16 * C + B * N_PTS * 24
    n_evals = int(sum(r["n_evals"] for r in res))

    # the same launch with memoisation off: every point's texel re-read at every evaluation,
    # i.e. the reference's data movement -- the HBM-bound form of the loop
    nm = {}
    if not args.no_nomemo:
        opts_nm = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=args.wgs,
                                  memoize=False)
        batch_nm = rf.AsyncBatch(probs, opts_nm)
        batch_nm.launch()
        torch.cuda.synchronize()
        s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(1, min(args.steps, 5))
        s_ev.record(stream)
        for _ in range(reps):
            batch_nm.launch()
        e_ev.record(stream)
        torch.cuda.synchronize()
        nm_s = s_ev.elapsed_time(e_ev) / reps / 1e3
        res_nm = batch_nm.results()
        same = all(np.array_equal(a["R"], b["R"]) and np.array_equal(a["t"], b["t"]) for a, b in zip(res, res_nm))
        nm_bytes = int(sum(r["texel_gathers"] for r in res_nm)) * 16 * C + B * N_PTS * 24
        nm = {"ms_per_launch": round(nm_s * 1e3, 4), "pose_refinements_per_s": round(B / nm_s, 1),
              "gathered_bytes_per_launch": nm_bytes, "achieved_GB_per_s": round(nm_bytes / nm_s / 1e9, 1),
              "frac": round(nm_bytes / nm_s / HBM_PEAK, 4), "poses_bit_identical_to_memoised": bool(same)}
        del batch_nm

    # FMPNP_LAYOUT_F: the same queries with only the f plane in HBM (the LM gather forms the
    # Sobel gradients), plus that layout's pack kernel (a channels-last copy)
    lf = {}
    if not args.no_layout_f:
        keep_f = []
        for q in range(B):
            inp = synth.problem_inputs(N_PTS, C, HF, WF, seed=rank * 100003 + q, device=dev)
            feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev, layout="f")
            keep_f.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"],
                                          inp["im_height"], inp["R0"], inp["t0"]))
            del inp
        batch_f = rf.AsyncBatch(keep_f, opts)
        batch_f.launch()
        torch.cuda.synchronize()
        s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(1, min(args.steps, 5))
        s_ev.record(stream)
        for _ in range(reps):
            batch_f.launch()
        e_ev.record(stream)
        torch.cuda.synchronize()
        f_s = s_ev.elapsed_time(e_ev) / reps / 1e3
        res_f = batch_f.results()
        f_gath = int(sum(r["texel_gathers"] for r in res_f))
        lf = {"ms_per_launch": round(f_s * 1e3, 4), "pose_refinements_per_s": round(B / f_s, 1),
              "gathered_bytes_per_launch": f_gath * 40 * C + B * N_PTS * 24,
              "bytes_rule": "per texel gather 9 neighbours x 4C (f) + 4C fref; fp64 point",
              "max_rot_diff_vs_fgrad_rad": float(max(np.arccos(np.clip((np.trace(a["R"].T @ b["R"]) - 1) / 2, -1, 1))
                                                     for a, b in zip(res, res_f))),
              "statuses": sorted({r["status"] for r in res_f})}
        del batch_f, keep_f

    # bilinear sampling (extension, FMPNP_BILINEAR): every supported point reads its 2x2 taps
    # of f, gx, gy plus fref at every evaluation -- SURVEY.md 8d's N*(52C+24) bytes per GN
    # iteration, no memoisation: the bandwidth-bound form of the loop
    bil = {}
    if not args.no_bilinear:
        opts_b = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=args.wgs,
                                 sampling="bilinear")
        batch_b = rf.AsyncBatch(probs, opts_b)
        batch_b.launch()
        torch.cuda.synchronize()
        s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(1, min(args.steps, 3))
        s_ev.record(stream)
        for _ in range(reps):
            batch_b.launch()
        e_ev.record(stream)
        torch.cuda.synchronize()
        b_s = s_ev.elapsed_time(e_ev) / reps / 1e3
        res_b = batch_b.results()
        b_evals = int(sum(r["n_evals"] for r in res_b))
        b_bytes = b_evals * N_PTS * (52 * C + 24)  # every evaluation samples every point (upper bound)
        bil = {"ms_per_launch": round(b_s * 1e3, 4), "pose_refinements_per_s": round(B / b_s, 1),
               "gn_iters_per_s": round(B * ITERS / b_s, 1), "algorithmic_bytes_per_launch": b_bytes,
               "bytes_rule": "SURVEY.md 8d bilinear: N*(52C+24) per point-evaluation (4 taps x f,gx,gy + fref "
                             "fp32, fp64 point)",
               "achieved_GB_per_s": round(b_bytes / b_s / 1e9, 1), "frac": round(b_bytes / b_s / HBM_PEAK, 4),
               "statuses": sorted({r["status"] for r in res_b})}
        del batch_b

    extras = {}
    if rank == 0 and not args.no_extras:
        extras = run_extras(args, dev, probs, keep, opts, rf, _lib, synth)

    if rank == 0:
        traffic, traffic_kernel = load_traffic(B)
        out = {
            "metric": "pose-refinements/sec (N=512 pts, C=256, 240x320, 50 LM iters)",
            "value": round(value, 3),
            "unit": "pose-refinements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.global_batch > 0 else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8d: smoothed L2-normalised random hypercolumns, seeded points)",
            "config": {"workload": "configs[1] shape batched as configs[2]: B independent queries per GPU "
                                   "(B=128 x 8 GPUs = 1024)",
                       "points": N_PTS, "channels": C, "feature_map": f"{HF}x{WF}", "image": f"{4 * HF}x{4 * WF}",
                       "iters": ITERS, "loss": "geman_mcclure", "lambda0": 0.01, "texel_storage": "f32",
                       "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"query sharding x{world} (no collectives)",
                       "launch": launch},
            "gn_iters_per_s": round(value * ITERS, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                         "traffic": traffic,
                         "kernel": traffic_kernel or "fmpnp::lm_kernel<float, 2, false, false, true>",
                         "avg_kernel_ms": round(avg_kernel_s * 1e3, 4),
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "bytes_rule": "SURVEY.md 8d: B * iters * N*(16C+24) (f, gx, gy, fref fp32 at one "
                                       "texel + fp64 point per GN iteration)",
                         "gathered_bytes_per_launch": gathered_bytes,
                         "gathered_GB_per_s": round(gathered_bytes / avg_kernel_s / 1e9, 1),
                         "texel_gathers_per_point_eval": round(gathers / max(1, n_evals * N_PTS), 4),
                         "note": "achieved counts the reference's data movement; the kernel re-reads a "
                                 "texel only when a point's pixel changed (bit-identical), so achieved > "
                                 "peak is possible; gathered_* is what it actually reads, no_memo the "
                                 "HBM-bound form"},
            "no_memo": nm,
            "bilinear": bil,
            "layout_f": lf,
            "statuses": statuses,
        }
        out.update(extras)
        print(json.dumps(out), flush=True)
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


def load_traffic(B):
    """(HBM bytes per launch, kernel name) from the committed rocprofv3 PMC summary of this
    workload (profiles/pmc_traffic.json, tools/gpu_profile.sh), if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("batch") == B:
            name = (d.get("kernel") or "").replace("void ", "").replace("(fmpnp::LaunchArgs)", "")
            return d.get("hbm_bytes_per_launch"), name or None
    except (OSError, ValueError):
        pass
    return None, None


def run_extras(args, dev, probs, keep, opts, rf, _lib, synth):
    out = {}
    # single-query latency: one query, workgroups of a team cooperate on its points
    one = rf.AsyncBatch(probs[:1], opts)
    for _ in range(3):
        one.launch()
    torch.cuda.synchronize()
    reps = 20
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        one.launch()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    out["single_query"] = {"ms_per_refinement": round(ms, 4), "gn_iters_per_s": round(ITERS / (ms / 1e3), 1),
                           "launch": _lib.last_launch()}
    # feature pack kernel (fused Sobel + channels-last): 4C bytes read + 12C written per texel.
    # Rotates over NP distinct maps and output buffers (NP x 314.6 MB > the 256 MB Infinity
    # Cache) so every launch streams from / to HBM.
    import ctypes
    L = _lib.load()
    st = _lib.stream_ptr(dev)
    NP = 4
    fms = [synth.feature_map(C, HF, WF, 777 + i, dev) for i in range(NP)]
    outs = [torch.empty((HF, WF, 3, C), dtype=torch.float32, device=dev) for _ in range(NP)]

    def pack(i):
        rc = L.fmpnp_pack_features(ctypes.c_void_p(fms[i % NP].data_ptr()), None, None, _lib.F32, C, HF, WF,
                                   ctypes.c_void_p(outs[i % NP].data_ptr()), _lib.F32, C, 0, 0, st)
        _lib.check(rc, "pack")
    for i in range(NP):
        pack(i)
    torch.cuda.synchronize()
    reps = 8 * NP
    s.record(torch.cuda.current_stream(dev))
    for i in range(reps):
        pack(i)
    e.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    pms = s.elapsed_time(e) / reps
    pbytes = 16 * C * HF * WF
    out["pack"] = {"ms": round(pms, 4), "GB_per_s": round(pbytes / (pms / 1e3) / 1e9, 1),
                   "frac_of_peak": round(pbytes / (pms / 1e3) / HBM_PEAK, 4),
                   "bytes_rule": "16C per texel (4C read + 12C written), %d distinct maps rotated" % NP}
    # the f-only layout's pack (FMPNP_LAYOUT_F): a channels-last copy, 4C read + 4C written
    outs_f = [torch.empty((HF, WF, C), dtype=torch.float32, device=dev) for _ in range(NP)]

    def pack_f(i):
        rc = L.fmpnp_pack_features_f(ctypes.c_void_p(fms[i % NP].data_ptr()), _lib.F32, C, HF, WF,
                                     ctypes.c_void_p(outs_f[i % NP].data_ptr()), _lib.F32, C, st)
        _lib.check(rc, "pack_f")
    for i in range(NP):
        pack_f(i)
    torch.cuda.synchronize()
    s.record(torch.cuda.current_stream(dev))
    for i in range(reps):
        pack_f(i)
    e.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    fms_ = s.elapsed_time(e) / reps
    fbytes = 8 * C * HF * WF
    out["pack_f"] = {"ms": round(fms_, 4), "GB_per_s": round(fbytes / (fms_ / 1e3) / 1e9, 1),
                     "frac_of_peak": round(fbytes / (fms_ / 1e3) / HBM_PEAK, 4),
                     "bytes_rule": "8C per texel (4C read + 4C written), %d distinct maps rotated" % NP}
    del outs_f
    del fms, outs
    # end to end from CHW hypercolumns (fmpnp.pipeline.RefinePipeline): pack + reference
    # gather + LM per batch, preparation of batch i+1 on a second stream under batch i's LM
    if not args.no_pipeline:
        import fmpnp
        from fmpnp.pipeline import RefinePipeline
        nb, qb = 4, 64
        batches, img = synth.pipeline_queries(nb, qb, N_PTS, C, HF, WF, device=dev, seed0=5000)
        pipe = RefinePipeline(img, storage=torch.float32, depth=2,
                              model_kwargs=dict(n_iters=ITERS, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                                ratio_threshold=None))
        pipe.run(batches)  # sizes the slab ring
        best = None
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = pipe.run(batches)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        out["end_to_end"] = {"queries_per_s": round(nb * qb / best, 1), "ms_per_query": round(best / (nb * qb) * 1e3, 4),
                             "batches": nb, "batch": qb,
                             "statuses": sorted({r["status"] for b in res for r in b}),
                             "note": "wall clock, host included: Sobel+pack and reference gather of every "
                                     "query (distinct maps) + one LM launch per batch, two streams"}
        del batches, pipe
    # CPU baseline: the oracle (C restatement of the reference loop), OpenMP over queries
    if args.cpu_sample > 0 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        out["cpu_baseline"] = cpu_baseline(args, keep[0])
    return out


def cpu_baseline(args, inp0):
    import oracle.oracle as orc
    threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    n_maps = min(threads, args.cpu_sample)
    from fmpnp import synth
    maps = []
    for m in range(n_maps):
        inp = synth.problem_inputs(N_PTS, C, HF, WF, seed=900000 + m, device="cpu")
        fm = inp["fmap"].double().numpy()
        gx, gy = orc.sobel(fm)
        maps.append((inp, fm, gx, gy))
    probs = []
    for q in range(args.cpu_sample):
        inp, fm, gx, gy = maps[q % n_maps]
        probs.append(orc.make_problem(inp["pts3d"], inp["fref"].double().numpy(), fm, gx, gy, inp["K"],
                                      inp["im_width"], inp["im_height"], inp["R0"], inp["t0"]))
    opts = orc.make_options(ITERS, 0.01, "geman_mcclure")
    orc.lib()
    t = time.perf_counter()
    orc.forward_batch(probs, opts, threads)
    dt = time.perf_counter() - t
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(args.cpu_sample / dt, 4), "unit": "pose-refinements/s", "cores": threads,
            "kind": "port", "gn_iters_per_s": round(args.cpu_sample * ITERS / dt, 1),
            "sample": f"{args.cpu_sample} cfg2 queries ({n_maps} distinct maps), 50 iters each, fp64 CHW "
                      f"reference layout, {dt:.1f}s", "cpu": cpu_model}


if __name__ == "__main__":
    main()
