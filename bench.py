#!/usr/bin/env python3
"""Benchmark: feature-metric PnP pose-refinements/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1] shape, batched as configs[2]): every GPU refines its
share of independent queries, each N=512 points, C=256 channels, 240x320 hypercolumn
(960x1280 image, stride 4), Geman-McClure, lambda0=0.01, 50 LM iterations, fp32 texels /
fp64 arithmetic.  Synthetic inputs (SURVEY.md §8d recipe; no dataset or CNN weights
offline).  One step = one launch of the LM kernel over the rank's whole batch (all 50
iterations of all its queries) with the packed features already resident in HBM.

Multi-GPU: the queries of a rank are fmpnp.shard.query_indices (the
global query index also seeds its inputs), timing is fmpnp.shard.timed_steps (barrier +
synchronise on both sides, max over ranks) -- the same code the gloo tests exercise.
Default: weak scaling, --batch 128 queries per GPU (configs[2]'s 1024 queries at 8 GPUs);
--global-batch 1024 is the fixed-total (strong) form.  No collective on the data path.

Roofline (dominant kernel = the LM launch): `achieved` = HBM bytes per launch from the
committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this exact workload
(profiles/rNN_pmc_<tag>.json of the newest round, tools/gpu_profile.sh; FETCH_SIZE doubled per
MI355X_MICROARCH.md) ÷ the launch time measured here with HIP events; without a matching
profile, the bytes the kernel's gathers move (counted live: texel gathers x 16C + the
fp64 points).  SURVEY.md §8d's reference-equivalent figure (every point re-read every
iteration) is reported separately as `reference_equivalent_GBps`: memoised gathers make
it exceed the HBM peak, so it is not a roofline fraction.

Legs reported beside the headline (rank 0): single query (configs[1]), the fixed total of
1024 queries on one GPU (SURVEY.md §8e's N=1 point), the harder initialisation and the
ratio test (input_configs/full_robotcar_08.gin:40), memoisation off, bilinear sampling,
the f-only layout, the pack kernels, the end-to-end pipeline, and the CPU baselines (C
restatement of the reference loop, OpenMP over queries; vectorised PyTorch-CPU fp64
restatement at 1 thread and at every core of the job's share) on a bounded sample whose
poses are compared with the GPU's for the same queries.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       N > 1 outside a launcher: bench.py starts N rank processes itself (torch.distributed.run,
       127.0.0.1, a free port) before anything touches the GPU and exits with their status;
       rank 0 prints the line.  Under a launcher (WORLD_SIZE set) --gpus must equal WORLD_SIZE.
"""
import argparse
import contextlib
import gc
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

N_PTS, C, HF, WF, ITERS = 512, 256, 240, 320, 50
HBM_PEAK = 8.0e12  # MI355X HBM3E spec (MI355X_MICROARCH.md)
B_ITER = N_PTS * (16 * C + 24)  # SURVEY.md §8d bytes per GN iteration per query (every point re-read)
LEGS = ["single", "hard", "ratio", "no_spec", "no_memo", "bilinear", "layout_f", "pack", "facade", "pipeline",
        "fixed1024", "pyramid1664", "cpu"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30000)  # ~10 s timed: visible to a GPU-busy sampler
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128, help="queries per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="total queries split over the GPUs (strong scaling); 0 = --batch per GPU")
    ap.add_argument("--init", choices=["easy", "hard"], default="easy")
    ap.add_argument("--ratio", type=float, default=None, help="ratio-test threshold (model.py:324-336)")
    ap.add_argument("--no-memo", action="store_true", help="re-gather every texel at every evaluation")
    ap.add_argument("--no-spec", action="store_true", help="memoised without the speculative next-texel gathers")
    ap.add_argument("--sampling", choices=["nearest", "bilinear"], default="nearest")
    ap.add_argument("--layout", choices=["fgrad", "f"], default="fgrad")
    ap.add_argument("--wgs", type=int, default=0, help="workgroups per query (0 = planner)")
    ap.add_argument("--event-every", type=int, default=10,
                    help="bracket every n-th timed launch with HIP events (kernel duration for the roofline)")
    ap.add_argument("--legs", default="all", help="comma list of " + ",".join(LEGS) + ", or all / none")
    ap.add_argument("--cpu-sample", type=int, default=1024, help="problems in the C-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--detail", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="side file for every leg's full record (the stdout line carries one summary per leg)")
    a = ap.parse_args()
    a.legs = set(LEGS) if a.legs == "all" else set() if a.legs == "none" else set(a.legs.split(","))
    if a.legs - set(LEGS):
        ap.error(f"unknown legs {sorted(a.legs - set(LEGS))}")
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


LINE_MAX_BYTES = 6000  # the driver keeps the tail of stdout: the line must fit it whole
_HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "gn_iters_per_s", "roofline", "cpu_baseline", "statuses",
              "rehearsal")
_ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "avg_kernel_ms",
              "rocprof_avg_kernel_ms", "reference_equivalent_GBps")
_CONFIG_KEYS = ("workload", "points", "channels", "feature_map", "iters", "loss", "texel_storage", "init",
                "ratio_threshold", "layout", "batch_per_gpu", "global_batch", "parallelism", "ranks")
_MS_KEYS = ("ms_per_launch", "ms_per_refinement", "ms_per_call", "ms_per_batch", "ms_per_query", "ms")
_RATE_KEYS = ("pose_refinements_per_s", "queries_per_s", "calls_per_s", "gn_iters_per_s", "GB_per_s")


def write_detail(out, path):
    """Every leg's full record (launch plans, byte rules, per-level rooflines, ...) as a side
    file; returns {"path", "sha256", "bytes"} for the stdout line, or a reason it was not written."""
    import hashlib
    blob = json.dumps(out, indent=1, default=str).encode()
    try:
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "wb") as f:
            f.write(blob)
    except OSError as e:
        return {"path": None, "error": str(e)}
    return {"path": path, "sha256": hashlib.sha256(blob).hexdigest(), "bytes": len(blob)}


def _leg_summary_compact(d):
    """One leg -> {ms, rate, frac} (+ a bit-identity flag where the leg has one)."""
    s = {}
    for k in _MS_KEYS:
        if isinstance(d.get(k), (int, float)):
            s["ms"] = d[k]
            break
    for k in _RATE_KEYS:
        if isinstance(d.get(k), (int, float)):
            s["rate"] = d[k]
            s["rate_unit"] = k
            break
    roof = d.get("roofline")
    if isinstance(roof, dict) and roof.get("frac") is not None:
        s["frac"] = roof["frac"]
    elif isinstance(d.get("frac_of_peak"), (int, float)):
        s["frac"] = d["frac_of_peak"]
    for k in ("poses_bit_identical_to_headline", "identical_to_full_pack", "refills_per_run", "within_1e-4"):
        if k in d:
            s[k] = d[k]
    return s


def compact_line(out, detail_ref):
    """The driver's JSON line: the headline keys (metric, value, ..., roofline, cpu_baseline) and
    ONE summary per leg; the legs' full records stay in the side file named by `detail`."""
    line = {k: out[k] for k in _HEAD_KEYS if k in out}
    if isinstance(line.get("config"), dict):
        line["config"] = {k: line["config"][k] for k in _CONFIG_KEYS if k in line["config"]}
    if isinstance(line.get("roofline"), dict):
        r = line["roofline"]
        line["roofline"] = {k: r[k] for k in _ROOF_KEYS if k in r}
        src = r.get("achieved_source", "")
        line["roofline"]["source"] = src.split(" (")[0][:160]
    cb = out.get("cpu_baseline")
    if isinstance(cb, dict):
        c = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample", "gn_iters_per_s", "cpu") if k in cb}
        pv = cb.get("poses_vs_gpu") or {}
        c["poses_vs_gpu"] = {k: pv[k] for k in ("max_rot_diff_rad", "max_t_diff_m", "within_1e-4") if k in pv}
        c["pytorch_cpu_fp64"] = {k: v.get("value") for k, v in (cb.get("pytorch_cpu_fp64") or {}).items()}
        if isinstance(cb.get("cpu_twin"), dict):
            tw = cb["cpu_twin"]
            c["cpu_twin"] = {"value": tw.get("value"), "cores": tw.get("cores"),
                             "within_1e-4": (tw.get("poses_vs_gpu") or {}).get("within_1e-4")}
        line["cpu_baseline"] = c
    legs = {}
    for k, v in out.items():
        if k in _HEAD_KEYS or not isinstance(v, dict) or k in ("kernel_timing",):
            continue
        summary = _leg_summary_compact(v)
        if summary:
            legs[k] = summary
        for k2, v2 in v.items():  # one level of nested legs (full_pack, robotcar_1664, median_query_n295, ...)
            if isinstance(v2, dict) and any(m in v2 for m in _MS_KEYS + _RATE_KEYS):
                legs[f"{k}.{k2}"] = _leg_summary_compact(v2)
    line["legs"] = legs
    line["detail"] = detail_ref
    text = json.dumps(line)
    if len(text) > LINE_MAX_BYTES:  # never lose the headline to a long line: drop leg summaries last-first
        for k in list(legs)[::-1]:
            del legs[k]
            line["legs_dropped"] = line.get("legs_dropped", 0) + 1
            if len(json.dumps(line)) <= LINE_MAX_BYTES:
                break
    return line


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: run N ranks under torch.distributed.run
    (one process per GPU) as a CHILD process -- this process has not touched the GPU and never
    execs -- and return its exit status.  Rank 0's JSON line reaches stdout directly."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def workload_tag(B, init, ratio, memo, sampling, layout, spec=True):
    """Key of a workload in profiles/rNN_pmc_<tag>.json."""
    t = f"b{B}_{init}"
    if ratio is not None:
        t += f"_ratio{ratio:g}"
    if not memo:
        t += "_nomemo"
    if sampling != "nearest":
        t += "_" + sampling
    if layout != "fgrad":
        t += "_layout" + layout
    if memo and not spec:
        t += "_nospec"
    return t


PROFILE_ROUNDS = ("r06", "r05", "r04", "r03", "r02")  # newest first


def load_traffic(tag, kernel, digest, root=ROOT):
    """HBM bytes per launch of this workload from a committed rocprofv3 FETCH_SIZE / WRITE_SIZE
    summary (profiles/rNN_pmc_<tag>.json), accepted only when it was taken of the kernel
    specialisation this launch ran (`kernel`, e.g. fmpnp::lm_kernel<float, 2, false, false, 6>)
    AND with the sources the loaded library was built from (`digest`, fmpnp_build_info).
    Returns (bytes, kernel, rocprof avg ns, path, why-not): a profile of another variant, of an
    older build, or without a recorded digest is never used -- the roofline then counts the
    kernel's own gathered bytes and says why."""
    rejected = []
    for rnd in PROFILE_ROUNDS:
        path = os.path.join("profiles", f"{rnd}_pmc_{tag}.json")
        try:
            with open(os.path.join(root, path)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        name = (d.get("kernel") or "").replace("void ", "").replace("(fmpnp::LaunchArgs)", "").strip()
        if name != kernel:
            rejected.append(f"{path}: kernel {name or '?'} is not the launch's {kernel}")
        elif digest == "unknown" or d.get("source_digest") != digest:
            rejected.append(f"{path}: taken with sources {d.get('source_digest')}, the loaded library is {digest}")
        elif not d.get("hbm_bytes_per_launch"):
            rejected.append(f"{path}: no FETCH/WRITE bytes")
        else:
            return d["hbm_bytes_per_launch"], name, d.get("kernel_avg_ns"), path, None
    return None, None, None, None, ("; ".join(rejected) or f"no profiles/rNN_pmc_{tag}.json")


def gather_bytes_rule(sampling, layout):
    """Bytes one texel gather moves (fp32) and the rule's text."""
    if layout == "f":
        return 40 * C, "9 neighbour texels x 4C (f) + 4C fref per gather"
    if sampling == "bilinear":
        return 52 * C, "4 taps x (f, gx, gy) 4C + 4C fref per sampled cell"
    return 16 * C, "(f, gx, gy, fref) x 4C per gather"


def roofline(tag, res, kernel_s, B, sampling, layout, launch):
    from fmpnp import _lib
    per_gather, rule = gather_bytes_rule(sampling, layout)
    gathers = int(sum(r["texel_gathers"] for r in res))
    n_evals = int(sum(r["n_evals"] for r in res))
    gathered = gathers * per_gather + B * N_PTS * 24
    kernel = _lib.kernel_name(launch)
    digest = _lib.library_digest()
    traffic, kname, prof_ns, prof_path, why_not = load_traffic(tag, kernel, digest)
    ach_bytes = traffic if traffic else gathered
    ach = ach_bytes / kernel_s
    return {"bound": "hbm", "achieved": round(ach / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK, 4), "traffic": traffic,
            "achieved_source": ("rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, %s (kernel and source digest %s match "
                                "this launch)" % (prof_path, digest)) if traffic
            else "LIVE gathered bytes (texel gathers counted by the kernel x bytes per gather): no committed PMC "
                 "profile of this kernel and build (%s)" % why_not,
            "kernel": kernel, "source_digest": digest, "avg_kernel_ms": round(kernel_s * 1e3, 4),
            "rocprof_avg_kernel_ms": round(prof_ns / 1e6, 4) if prof_ns else None,
            "gathered_bytes_per_launch": gathered, "gathered_GB_per_s": round(gathered / kernel_s / 1e9, 1),
            "gathered_bytes_rule": rule + " + 24 B fp64 point per query point",
            "texel_gathers_per_point_eval": round(gathers / max(1, n_evals * N_PTS), 4),
            "reference_equivalent_GBps": round(B * ITERS * B_ITER / kernel_s / 1e9, 1),
            "reference_equivalent_rule": "SURVEY.md 8d: B * iters * N*(16C+24) -- every point's texel re-read at "
                                         "every iteration, as the reference does; not a roofline fraction"}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))  # before any torch.cuda / HIP call
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"[bench] error: --gpus {args.gpus} but the launcher started {world} ranks (WORLD_SIZE)")
        sys.exit(2)
    dryrun = bool(os.environ.get("FMPNP_BENCH_DRYRUN"))  # CPU test of the launch path: touch no GPU
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # one process per GPU; FMPNP_BENCH_BACKEND=gloo (and more ranks than GPUs) rehearses the
    # distributed path on a one-GPU box -- the timing barrier and max-over-ranks only, reported as
    # a rehearsal with n_gpus = the distinct devices used (never a multi-GPU figure)
    backend = os.environ.get("FMPNP_BENCH_BACKEND", "nccl")
    # (device_count() does not initialise the GPU on this image; FMPNP_BENCH_NDEV: dry runs only)
    ndev = (int(os.environ.get("FMPNP_BENCH_NDEV", "1")) if dryrun else 0) or max(1, torch.cuda.device_count())
    if dist and backend == "nccl" and world > ndev:
        log(f"[bench] error: {world} ranks but {ndev} visible GPU(s): one process per GPU (rehearse more ranks "
            f"with FMPNP_BENCH_BACKEND=gloo)")
        sys.exit(3)
    gpu = local % ndev
    if dryrun:
        from fmpnp import shard as _sh
        n_gpus, rpd = _sh.device_accounting([r % ndev for r in range(world)])  # single node: LOCAL_RANK = RANK
        print(json.dumps({"rank": rank, "world": world, "device": gpu, "n_gpus": n_gpus, "ranks": world,
                          "ranks_per_device": rpd,
                          "queries": list(_sh.query_indices(rank, world, per_rank=args.batch,
                                                            global_batch=args.global_batch))}), flush=True)
        return
    if dist:
        import torch.distributed as tdist
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            tdist.init_process_group(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    from fmpnp import _lib, refine as rf, shard, synth

    # ---------------- setup (untimed): this rank's queries, packed in HBM ----------------
    qidx = shard.query_indices(rank, world, per_rank=args.batch, global_batch=args.global_batch)
    B = len(qidx)
    memo = not args.no_memo
    t0 = time.time()
    feats, inputs, probs = [], [], []
    for q in qidx:
        inp = synth.problem_inputs(N_PTS, C, HF, WF, seed=q, device=dev, init=args.init)
        f = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev, layout=args.layout)
        probs.append(rf.make_problem(f, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                     inp["R0"], inp["t0"]))
        feats.append(f)
        inp.pop("fmap")
        inputs.append(inp)
    torch.cuda.synchronize()
    if rank == 0:
        log(f"[bench] setup {B} queries/GPU in {time.time() - t0:.1f}s "
            f"({torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB resident)")
    opts = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, ratio_threshold=args.ratio, dtype=_lib.F32,
                           wgs_per_problem=args.wgs, memoize=memo, sampling=args.sampling,
                           speculate=not args.no_spec)
    batch = rf.AsyncBatch(probs, opts)

    # ---------------- warmup ----------------
    for _ in range(args.warmup):
        batch.launch()
    torch.cuda.synchronize()
    launch = _lib.last_launch()

    # ---------------- timed region: exactly K launches ----------------
    # HIP events bracket every `event_every`-th launch (the per-launch kernel duration of the
    # roofline); the others run back to back with nothing between them
    stream = torch.cuda.current_stream(dev)  # the stream the launches go to (_lib.stream_ptr)
    every = max(1, args.event_every)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range((args.steps + every - 1) // every)]

    def step(k):
        if k % every:
            batch.launch()
            return
        e0, e1 = ev[k // every]
        e0.record(stream)
        batch.launch()
        e1.record(stream)

    elapsed = shard.timed_steps(step, args.steps, device=dev)
    props = torch.cuda.get_device_properties(dev)
    my_dev = (__import__("socket").gethostname(), getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", gpu),
              getattr(props, "pci_device_id", 0))
    n_gpus, ranks_per_device = shard.device_accounting(shard.gather_device_ids(my_dev))
    kernel_s = float(np.mean([a.elapsed_time(b) for a, b in ev])) / 1e3
    res = batch.results()
    statuses = sorted({r["status"] for r in res})
    if any(s & _lib.STATUS_SYNC_TIMEOUT for s in statuses):
        raise RuntimeError("sync timeout in the LM kernel")
    # every rank's queries: the fixed total (strong scaling), else the per-rank batch on each rank
    total = args.global_batch if args.global_batch > 0 else args.batch * world
    value = total * args.steps / elapsed
    tag = workload_tag(B, args.init, args.ratio, memo, args.sampling, args.layout, not args.no_spec)

    extras = {}
    if rank == 0 and args.legs:
        extras = run_legs(args, dev, probs, feats, inputs, opts, res, rf, _lib, synth)

    if rank == 0:
        out = {
            "metric": "pose-refinements/sec (N=512 pts, C=256, 240x320, 50 LM iters)",
            "value": round(value, 3),
            "unit": "pose-refinements/s",
            "n_gpus": n_gpus,  # distinct devices used (ranks sharing a GPU count once)
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.global_batch > 0 else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8d: smoothed L2-normalised random hypercolumns, seeded points; "
                    "seed = global query index)",
            "config": {"workload": "configs[1] shape batched as configs[2]: "
                                   + (f"{args.global_batch} queries split over the GPUs" if args.global_batch
                                      else f"{args.batch} independent queries per GPU (x8 GPUs = 1024)"),
                       "points": N_PTS, "channels": C, "feature_map": f"{HF}x{WF}", "image": f"{4 * HF}x{4 * WF}",
                       "iters": ITERS, "loss": "geman_mcclure", "lambda0": 0.01, "texel_storage": "f32",
                       "init": args.init, "ratio_threshold": args.ratio, "memoised": memo,
                       "speculative_gathers": memo and not args.no_spec and _lib.spec_build(),
                       "sampling": args.sampling, "layout": args.layout,
                       "batch_per_gpu": B, "global_batch": total,
                       "parallelism": f"query sharding x{world} (no collectives)", "launch": launch,
                       "ranks": world, "ranks_per_device": ranks_per_device, "devices_visible": ndev,
                       "backend": (backend if dist else None)},
            "gn_iters_per_s": round(value * ITERS, 1),
            "roofline": roofline(tag, res, kernel_s, B, args.sampling, args.layout, launch),
            "kernel_timing": f"HIP events on the launch stream around every {every}-th of the {args.steps} timed "
                             f"launches ({len(ev)} samples)",
            "statuses": statuses,
        }
        if ranks_per_device > 1:
            out["rehearsal"] = (f"{world} ranks on {n_gpus} device(s): a rehearsal of the distributed path "
                                f"(barrier + max-over-ranks timing), not a multi-GPU scaling figure")
        out.update(extras)
        ref = write_detail(out, args.detail)
        print(json.dumps(compact_line(out, ref)), flush=True)
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


def time_launches(batch, reps, stream, warmup=1):
    """Mean ms per launch over `reps` back-to-back launches (after `warmup` launches), results."""
    for _ in range(warmup):
        batch.launch()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(reps):
        batch.launch()
    e.record(stream)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps, batch.results()


def rot_angle(Ra, Rb):
    c = (np.trace(np.asarray(Ra).T @ np.asarray(Rb)) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


def leg_summary(tag, ms, res, B, sampling="nearest", layout="fgrad", base=None):
    """(call right after the leg's launches: its roofline matches profiles against last_launch())"""
    from fmpnp import _lib
    rf_s = B / (ms / 1e3)
    d = {"ms_per_launch": round(ms, 4), "pose_refinements_per_s": round(rf_s, 1),
         "gn_iters_per_s": round(rf_s * ITERS, 1), "statuses": sorted({r["status"] for r in res}),
         "roofline": roofline(tag, res, ms / 1e3, B, sampling, layout, _lib.last_launch())}
    if base is not None:
        d["max_rot_diff_vs_headline_rad"] = float(max(rot_angle(a["R"], b["R"]) for a, b in zip(res, base)))
        d["poses_bit_identical_to_headline"] = bool(all(np.array_equal(a["R"], b["R"]) and
                                                        np.array_equal(a["t"], b["t"]) for a, b in zip(res, base)))
    return d


def run_legs(args, dev, probs, feats, inputs, opts, res_main, rf, _lib, synth):
    out = {}
    stream = torch.cuda.current_stream(dev)
    B = len(probs)
    memo = not args.no_memo

    def opt(**kw):
        base = dict(ratio_threshold=args.ratio, dtype=_lib.F32, wgs_per_problem=args.wgs, memoize=memo,
                    sampling=args.sampling)
        base.update(kw)
        return rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, **base)

    if "single" in args.legs:  # configs[1]: one query, one launch
        ms, r1 = time_launches(rf.AsyncBatch(probs[:1], opts), 20, stream)
        out["single_query"] = {"ms_per_refinement": round(ms, 4), "gn_iters_per_s": round(ITERS / (ms / 1e3), 1),
                               "launch": _lib.last_launch()}
    # the harder initialisation (golden vectors' perturbation): same maps, other start poses
    if "hard" in args.legs and args.init == "easy":
        R0, t0 = synth.INITS["hard"]
        hp = [rf.make_problem(p.feats, p.fref, p.pts3d, p.K, p.im_width, p.im_height, R0, t0) for p in probs]
        ms, r = time_launches(rf.AsyncBatch(hp, opts), 10, stream)
        out["hard_init"] = leg_summary(workload_tag(B, "hard", args.ratio, memo, args.sampling, args.layout),
                                       ms, r, B, args.sampling, args.layout)
        if "ratio" in args.legs:
            ms, r = time_launches(rf.AsyncBatch(hp, opt(ratio_threshold=0.8)), 10, stream)
            out["hard_init_ratio08"] = leg_summary(workload_tag(B, "hard", 0.8, memo, args.sampling, args.layout),
                                                   ms, r, B, args.sampling, args.layout)
            out["hard_init_ratio08"]["kernel_variant"] = "RATIO=true"
        del hp
    if "ratio" in args.legs and args.ratio is None:  # input_configs/full_robotcar_08.gin:40
        ms, r = time_launches(rf.AsyncBatch(probs, opt(ratio_threshold=0.8)), 10, stream)
        out["ratio08"] = leg_summary(workload_tag(B, args.init, 0.8, memo, args.sampling, args.layout), ms, r, B,
                                     args.sampling, args.layout)
        out["ratio08"]["kernel_variant"] = "RATIO=true"
    if "no_spec" in args.legs and memo and _lib.spec_build():  # memoised, without the speculative gathers
        ms, r = time_launches(rf.AsyncBatch(probs, opt(speculate=False)), 10, stream)
        out["no_spec"] = leg_summary(workload_tag(B, args.init, args.ratio, memo, args.sampling, args.layout, False),
                                     ms, r, B, args.sampling, args.layout, base=res_main)
    if "bilinear" in args.legs and args.sampling == "nearest" and args.layout == "fgrad":  # extension
        # the cell memo (default); direct sampling of every point at every evaluation runs in the
        # 1024-query leg below (an HBM-streamed working set)
        ms, r = time_launches(rf.AsyncBatch(probs, opt(sampling="bilinear")), 10, stream)
        out["bilinear"] = leg_summary(workload_tag(B, args.init, args.ratio, memo, "bilinear", "fgrad"), ms, r, B,
                                      "bilinear", "fgrad")
        out["bilinear"]["launch"] = _lib.last_launch()
    if "layout_f" in args.legs and args.layout == "fgrad" and args.sampling == "nearest":
        fp = []
        for q, inp in enumerate(inputs):
            fm = synth.feature_map(C, HF, WF, q, dev)  # rank 0: query q has global index (seed) q
            ff = rf.pack_features(fm, storage=torch.float32, device=dev, layout="f")
            fp.append(rf.make_problem(ff, probs[q].fref, probs[q].pts3d, inp["K"], inp["im_width"],
                                      inp["im_height"], inp["R0"], inp["t0"]))
            del fm
        ms, r = time_launches(rf.AsyncBatch(fp, opts), 5, stream)
        out["layout_f"] = leg_summary(workload_tag(B, args.init, args.ratio, memo, "nearest", "f"), ms, r, B,
                                      "nearest", "f", base=res_main)
        del fp
    if "pack" in args.legs:
        out.update(pack_legs(dev, _lib, synth))
    if "facade" in args.legs:
        out["facade_call"] = facade_leg(dev, synth)
    if "pipeline" in args.legs:
        out["end_to_end"] = pipeline_leg(dev, synth)
    if "pyramid1664" in args.legs:
        out["pyramid_robotcar_1664"] = pyramid_legs(dev, rf, synth, _lib, stream)
    if ({"fixed1024", "no_memo", "bilinear"} & args.legs) and B < 1024 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        out.update(fixed_total_leg(args, dev, probs, feats, inputs, opts, rf, synth, stream, opt))
    if "cpu" in args.legs and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        out["cpu_baseline"] = cpu_baseline(args, res_main, synth, dev)
    return out


def fixed_total_leg(args, dev, probs, feats, inputs, opts, rf, synth, stream, opt):
    """The 1024-query set resident on ONE GPU (the headline's queries plus the next ones by global
    index; packed layout when it fits in HBM, 1024 x 236 MB, else the f-only layout):
      fixed_total_1024   SURVEY.md §8e's fixed total of 1024 on one GPU (the N = 1 point of the
                         strong-scaling curve), memoised, one launch;
      no_memo            every point's texel re-read at every evaluation (the reference's data
                         movement), the same 1024 queries;
      bilinear_direct    bilinear sampling of every supported point at every evaluation.
    The last two stream a working set of >= 2 GB per launch, far beyond the 256 MB Infinity Cache,
    so their traffic is HBM traffic (at B = 128 their per-launch working set is about the cache's
    size and part of it was served from there)."""
    from fmpnp import _lib
    n = 1024
    torch.cuda.synchronize()
    # the earlier legs' pipelines and façade buffers (reference cycles: freed by the collector)
    gc.collect()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(dev)
    need = (n - len(probs)) * (HF * WF * 3 * C * 4 + N_PTS * C * 4 + N_PTS * 24) + (8 << 30)
    layout = args.layout if free > need else "f"
    if layout != args.layout:
        print(f"[bench] fixed_total_1024: {free / 2**30:.1f} GiB free < {need / 2**30:.1f} GiB needed for the "
              f"{args.layout} layout: f-only layout", file=sys.stderr)
    if layout != args.layout:
        probs, feats = [], []
    ps = list(probs)
    for q in range(len(ps), n):
        inp = synth.problem_inputs(N_PTS, C, HF, WF, seed=q, device=dev, init=args.init)
        f = rf.pack_features(inp["fmap"], storage=torch.float32, device=dev, layout=layout)
        ps.append(rf.make_problem(f, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                  inp["R0"], inp["t0"]))
        del inp
    out = {}
    memo = not args.no_memo
    # (226 GB of freshly allocated maps: the first launches also warm the address translation)
    ms, r = time_launches(rf.AsyncBatch(ps, opts), 20, stream, warmup=3)
    if "fixed1024" in args.legs:
        d = leg_summary(workload_tag(n, args.init, args.ratio, memo, args.sampling, layout), ms, r, n,
                        args.sampling, layout)
        d.update(layout=layout, launch=_lib.last_launch(),
                 resident_GiB=round(torch.cuda.memory_allocated(dev) / 2**30, 1),
                 free_GiB_before=round(free / 2**30, 1), packed_need_GiB=round(need / 2**30, 1))
        out["fixed_total_1024"] = d
    note = ("1024 queries resident: >= 2 GB of distinct texels per launch, beyond the 256 MB Infinity Cache "
            "(HBM-streamed)")
    if "no_memo" in args.legs and memo and layout == "fgrad":
        ms2, r2 = time_launches(rf.AsyncBatch(ps, opt(memoize=False)), 3, stream)
        d = leg_summary(workload_tag(n, args.init, args.ratio, False, args.sampling, layout), ms2, r2, n,
                        args.sampling, layout, base=r)
        d.update(launch=_lib.last_launch(), working_set=note)
        out["no_memo"] = d
    if "bilinear" in args.legs and args.sampling == "nearest" and layout == "fgrad":
        ms3, r3 = time_launches(rf.AsyncBatch(ps, opt(sampling="bilinear", memoize=False)), 2, stream)
        d = leg_summary(workload_tag(n, args.init, args.ratio, False, "bilinear", "fgrad"), ms3, r3, n, "bilinear",
                        "fgrad")
        d.update(launch=_lib.last_launch(), working_set=note)
        out["bilinear_direct"] = d
    del ps
    torch.cuda.empty_cache()
    return out


def pyramid_legs(dev, rf, synth, _lib, stream):
    """The production pyramid at the largest (866) and the median (295) num_final_matches of
    results/results_s2dhm/robotcar/summary.csv (column 5): the typical query and the worst one."""
    out = pyramid_leg(dev, rf, synth, _lib, stream, N=866)
    out["median_query_n295"] = pyramid_leg(dev, rf, synth, _lib, stream, N=295)
    return out


def pyramid_level_roofline(N, li, ms, gathers, C_level, root=ROOT):
    """One pyramid level against the HBM roofline: HBM bytes per launch from the committed
    rocprofv3 FETCH/WRITE summary (profiles/rNN_pmc_pyramid_n<N>.json, tools/gpu_profile_pyramid.sh)
    taken with the loaded library's sources, else the live gathered bytes (gathers x 16 C + points)."""
    from fmpnp import _lib
    digest = _lib.library_digest()
    for rnd in PROFILE_ROUNDS:
        path = os.path.join("profiles", f"{rnd}_pmc_pyramid_n{N}.json")
        try:
            with open(os.path.join(root, path)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if digest != "unknown" and d.get("source_digest") == digest:
            lv = d["levels"][li]
            b = lv["hbm_bytes_per_launch"]
            return {"bound": "hbm", "achieved": round(b / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK / 1e9,
                    "unit": "GB/s", "frac": round(b / (ms / 1e3) / HBM_PEAK, 4), "traffic": b,
                    "source": f"{path} (rocprofv3 {lv['kernel_avg_ns'] / 1e6:.4f} ms, {lv['kernel']})"}
    b = gathers * 16 * C_level + 32 * N * 24
    return {"bound": "hbm", "achieved": round(b / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": round(b / (ms / 1e3) / HBM_PEAK, 4), "traffic": None,
            "source": "LIVE gathered bytes (texel gathers x 16C + fp64 points): no committed PMC profile of this build"}


def pyramid_leg(dev, rf, synth, _lib, stream, B=32, N=866):
    """The reference's production refinement: RobotCar hypercolumns of C = 1664 channels
    (network.gin:18) at 256x256 for a 1024x1024 image, N points per query (866: the largest
    num_final_matches of results/results_s2dhm/robotcar/summary.csv; 295: its median),
    Geman-McClure, 50 iterations per level over the channel pyramid of
    input_configs/default_robotcar.gin:75 [(640,1664), (128,640), (0,128)] (multilevel_optimization,
    model.py:178-213).  B queries per launch, one launch per level, each level starting from the
    previous level's poses.  The planner's workgroups per query (G, each level's `launch`): 32 queries
    leave 224 of the 256 CUs idle; a query of more than eight 64-point blocks (N = 866: 14) is spread
    over G = 8 workgroups -- the fastest of G = 1, 2, 4, 8 measured at N = 866
    (profiles/r03_pyramid1664_g_sweep.txt) --, one of at most eight (N = 295: 5 blocks) keeps G = 1,
    where a member's exchange costs more than its share of the evaluation saves (fmpnp_api.hip)."""
    levels = [(640, 1664), (128, 640), (0, 128)]
    torch.cuda.synchronize()
    feats, frefs, inps = [], [], []
    for q in range(B):
        inp = synth.problem_inputs(N, 1664, 256, 256, seed=20000 + q, device=dev, init="easy")
        feats.append(rf.pack_features(inp.pop("fmap"), storage=torch.float32, device=dev))
        frefs.append(inp.pop("fref"))
        inps.append(inp)
    R = [i["R0"] for i in inps]
    t = [i["t0"] for i in inps]
    opts = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
    per_level, total = [], 0.0
    for li, (cb, ce) in enumerate(levels):
        ps = [rf.make_problem(feats[q], frefs[q], inps[q]["pts3d"], inps[q]["K"], inps[q]["im_width"],
                              inps[q]["im_height"], R[q], t[q], c_begin=cb, c_end=ce) for q in range(B)]
        ms, res = time_launches(rf.AsyncBatch(ps, opts), 10, stream)
        total += ms
        gathers = sum(r["texel_gathers"] for r in res)
        per_level.append({"channels": [cb, ce], "ms_per_launch": round(ms, 4), "launch": _lib.last_launch(),
                          "statuses": sorted({r["status"] for r in res}),
                          "texel_gathers_per_point_eval": round(gathers / max(1, N * sum(r["n_evals"] for r in res)),
                                                                4),
                          "roofline": pyramid_level_roofline(N, li, ms, gathers, ce - cb)})
        R = [r["R"] for r in res]
        t = [r["t"] for r in res]
    del feats, frefs
    torch.cuda.empty_cache()
    return {"queries": B, "points": N, "ms_per_batch": round(total, 4),
            "pose_refinements_per_s": round(B / (total / 1e3), 1), "levels": per_level,
            "workload": f"C=1664 256x256 hypercolumns, 1024x1024 image, {N} points, GM, 50 iters per level, "
                        "default_robotcar.gin:75 channel pyramid; sum of the three level launches"}


def pack_legs(dev, _lib, synth):
    """The feature-pack kernels (fused Sobel + channels-last; f-only copy), rotating over NP
    distinct maps and outputs (NP x 314.6 MB > the 256 MB Infinity Cache: HBM-streamed)."""
    import ctypes
    out = {}
    L = _lib.load()
    st = _lib.stream_ptr(dev)
    stream = torch.cuda.current_stream(dev)
    NP = 4
    fms = [synth.feature_map(C, HF, WF, 777 + i, dev) for i in range(NP)]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, planes, fn in (("pack", 3, L.fmpnp_pack_features), ("pack_f", 1, L.fmpnp_pack_features_f)):
        outs = [torch.empty((HF, WF, planes, C), dtype=torch.float32, device=dev) for _ in range(NP)]

        def run(i):
            if planes == 3:
                rc = fn(ctypes.c_void_p(fms[i % NP].data_ptr()), None, None, _lib.F32, C, HF, WF,
                        ctypes.c_void_p(outs[i % NP].data_ptr()), _lib.F32, C, 0, 0, st)
            else:
                rc = fn(ctypes.c_void_p(fms[i % NP].data_ptr()), _lib.F32, C, HF, WF,
                        ctypes.c_void_p(outs[i % NP].data_ptr()), _lib.F32, C, st)
            _lib.check(rc, name)
        for i in range(NP):
            run(i)
        torch.cuda.synchronize()
        reps = 8 * NP
        s.record(stream)
        for i in range(reps):
            run(i)
        e.record(stream)
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        nbytes = (4 + 4 * planes) * C * HF * WF
        out[name] = {"ms": round(ms, 4), "GB_per_s": round(nbytes / (ms / 1e3) / 1e9, 1),
                     "frac_of_peak": round(nbytes / (ms / 1e3) / HBM_PEAK, 4),
                     "bytes_rule": f"{4 + 4 * planes}C per texel (4C read + {4 * planes}C written), "
                                   f"{NP} distinct maps rotated"}
        del outs
    del fms
    return out


ROBOTCAR_PYRAMID = [(640, 1664, None, None), (128, 640, None, None), (0, 128, None, None)]  # default_robotcar.gin:75
FACADE_SHAPES = {  # name: (N, C, Hf, Wf, feature_pyramid, distinct queries cycled)
    "cfg2": (N_PTS, C, HF, WF, None, 8),
    "robotcar_n295": (295, 1664, 256, 256, ROBOTCAR_PYRAMID, 4),
    "robotcar_n866": (866, 1664, 256, 256, ROBOTCAR_PYRAMID, 4),
}


class _StubNet:
    """optimize_feature_pnp's `net` (s2dhm ImageRetrievalModel): compute_hypercolumn of the
    reference image returns its device hypercolumn (optimize_feature_pnp.py:78-82); the CNN is
    out of scope, so the map is the synthetic one already resident."""

    def __init__(self, ref_hc):
        self.ref_hc = ref_hc

    def compute_hypercolumn(self, names, to_cpu=False, resize=True):
        return self.ref_hc, None


def facade_queries(dev, synth, name, seed0=9000):
    N, Cq, H, W, pyr, nq = FACADE_SHAPES[name]
    (batch,), img = synth.pipeline_queries(1, nq, N, Cq, H, W, device=dev, seed0=seed0)
    return batch, img, pyr


def facade_calls(dev, synth, name, calls=24, warmup=2, via="feature_pnp", queries=None):
    """The reference consumer's own call, one query per call (sparse_to_dense_predictor.py:242-247
    times one optimize_feature_pnp call per query): the query hypercolumn [1, C, H, W] fp32 already
    on the device, a new model per call (gin builds one, optimize_feature_pnp.py:63), the pose back
    on the host.  via="optimize_feature_pnp" adds the stub net's reference hypercolumn and the
    quaternion (optimize_feature_pnp.py:73-91).  Wall clock per call over `calls` calls cycling
    through distinct queries."""
    import fmpnp
    from fmpnp import matrix_utils
    batch, img, pyr = queries or facade_queries(dev, synth, name)
    pred_t = __import__("collections").namedtuple(
        "Prediction", "points_3d reference_inliers matrix quaternion reference_filename inlier_mask")

    def one(i):
        q, r, p, K = batch[i % len(batch)]
        model = fmpnp.sparseFeaturePnP(n_iters=ITERS, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01)
        if via == "feature_pnp":
            R, t, model = fmpnp.feature_pnp(q[None], r, p, K, img, feature_pyramid=pyr, model=model)
            return model
        pr = pred_t(p.points_3d, p.reference_inliers, p.matrix, matrix_utils.matrix_quaternion(p.matrix),
                    "reference.png", None)
        # (the reference's "Initial : ..." / "Final : ..." prints stay in the timed call, on stderr: stdout
        # carries only the bench's one JSON line)
        with contextlib.redirect_stdout(sys.stderr):
            t, quat, model = fmpnp.optimize_feature_pnp(q[None], _StubNet(r), pr, K, image_shape=img,
                                                        feature_pyramid=pyr, model=model)
        return model
    from fmpnp import _lib
    for i in range(warmup):
        one(i)
    torch.cuda.synchronize()
    reruns0 = _lib.load().fmpnp_feature_pnp_reruns()
    t0 = time.perf_counter()
    statuses = set()
    for i in range(calls):
        m = one(i)
        statuses.add(int(m.status_ or 0))
    dt = time.perf_counter() - t0
    N, Cq, H, W = FACADE_SHAPES[name][:4]
    reruns = _lib.load().fmpnp_feature_pnp_reruns() - reruns0
    return {"ms_per_call": round(dt / calls * 1e3, 4), "calls_per_s": round(calls / dt, 1), "calls": calls,
            "window_reruns": int(reruns),
            "distinct_queries": len(batch), "statuses": sorted(statuses), "via": via,
            "shape": f"N={N} C={Cq} {H}x{W}" + (" pyramid default_robotcar.gin:75" if pyr else "")}


def facade_leg(dev, synth):
    """Per-call latency of the consumer's swap-in (verdict r04 item 2): feature_pnp at cfg2 and at
    the RobotCar production shape (C = 1664 @ 256x256, the median 295 and the largest 866 points,
    the channel pyramid), and optimize_feature_pnp with a stub net at cfg2."""
    out = {}
    for name in FACADE_SHAPES:
        qs = facade_queries(dev, synth, name)
        out[name] = facade_calls(dev, synth, name, queries=qs)
        if name == "cfg2":
            out["cfg2_optimize_feature_pnp"] = facade_calls(dev, synth, name, via="optimize_feature_pnp", queries=qs)
        del qs
        torch.cuda.empty_cache()
    return out


PIPE_WINDOW = 5  # texels around each point's initial texel that the end-to-end leg packs (fmpnp.pipeline window)


def pipeline_leg(dev, synth):
    """End to end from CHW hypercolumns (fmpnp.pipeline.RefinePipeline): pack + reference
    gather + LM per batch, preparation of batch i+1 on a second stream under batch i's LM.
    The leg's number is the windowed f-only pack (radius PIPE_WINDOW; a query that leaves its
    window is packed in full and refined again -- `refills`, bit-identical results either way,
    tests/test_window_pack.py); `full_pack` is the same workload with every texel packed."""
    import fmpnp
    from fmpnp.pipeline import RefinePipeline
    nb, qb = 4, 64
    batches, img = synth.pipeline_queries(nb, qb, N_PTS, C, HF, WF, device=dev, seed0=5000)

    def timed(window, batches=batches, steady=False):
        """Best of 3 runs of the nb batches (and, steady=True, of the same batches streamed twice on
        the SAME pipeline: the second four's rate, the fill and drain counted once)."""
        pipe = RefinePipeline(img, storage=torch.float32, depth=2, window=window,
                              model_kwargs=dict(n_iters=ITERS, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                                ratio_threshold=None))
        pipe.run(batches)  # sizes the slab ring
        best = {1: None, 2: None}
        res, refills = None, 0
        pipe.host_s = dict.fromkeys(pipe.host_s, 0.0)
        runs = 0
        for _ in range(3):
            for rep in ((1, 2) if steady else (1,)):
                before = pipe.refills
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = pipe.run(batches * rep)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                best[rep] = dt if best[rep] is None else min(best[rep], dt)
                runs += rep
                if rep == 1:
                    res, refills = r, max(refills, pipe.refills - before)
        host_ms = {k: round(v / runs * 1e3, 4) for k, v in pipe.host_s.items()}
        return nb * qb / best[1], best, res, refills, host_ms

    qps, best, res, refills, host_ms = timed(PIPE_WINDOW, steady=True)
    fqps, fbest, fres, _, _ = timed(None)
    d8 = best[2] - best[1]
    steady = nb * qb / d8 if d8 > 0.05 * best[1] else None  # (no figure from a difference within noise)
    same = all(np.array_equal(a["R"], b["R"]) and np.array_equal(a["t"], b["t"]) and a["best_cost"] == b["best_cost"]
               for x, y in zip(res, fres) for a, b in zip(x, y))
    hard, _ = synth.pipeline_queries(nb, qb, N_PTS, C, HF, WF, device=dev, seed0=5000, init="hard")
    hqps, hbest, _, hrefills, _ = timed(PIPE_WINDOW, batches=hard)
    del hard
    out = {"queries_per_s": round(qps, 1), "ms_per_query": round(best[1] / (nb * qb) * 1e3, 4),
           "batches": nb, "batch": qb, "statuses": sorted({r["status"] for b in res for r in b}),
           "window": PIPE_WINDOW, "refills_per_run": refills, "identical_to_full_pack": same,
           "steady_state_queries_per_s": round(steady, 1) if steady else None,
           "host_ms_per_pass_of_4": host_ms,
           "hard_init": {"queries_per_s": round(hqps, 1), "refills_per_run": hrefills,
                         "ms_per_query": round(hbest[1] / (nb * qb) * 1e3, 4)},
           "note": "wall clock, host included: windowed f-only pack and reference gather of every query (distinct "
                   "maps) + one LM launch per batch, two streams; steady state = the same pipeline streaming the "
                   "batches twice, the second pass's rate"}
    out["roofline"] = pipeline_roofline(qps, PIPE_WINDOW)
    out["full_pack"] = {"queries_per_s": round(fqps, 1), "ms_per_query": round(fbest[1] / (nb * qb) * 1e3, 4),
                        "roofline": pipeline_roofline(fqps, None)}
    del batches, timed  # (timed's defaults hold the batches too)
    out["robotcar_1664"] = robotcar_pipeline_leg(dev, synth)
    return out


def robotcar_pipeline_leg(dev, synth, nb=2, qb=32, N=866):
    """End to end at the RobotCar production shape: CHW hypercolumns of C = 1664 at 256x256
    (network.gin:18) for 1024x1024 images, N = 866 points (the largest num_final_matches of
    results/results_s2dhm/robotcar/summary.csv), the channel pyramid of
    input_configs/default_robotcar.gin:75 chained on the device (RefinePipeline levels), f-only
    pack (full: 866 windows cover most of a 256x256 map) + reference gather + three LM launches
    per batch of 32, preparation of the next batch under the current one's launches."""
    import fmpnp
    from fmpnp.pipeline import RefinePipeline
    batches, img = synth.pipeline_queries(nb, qb, N, 1664, 256, 256, device=dev, seed0=7000)
    pipe = RefinePipeline(img, storage=torch.float32, depth=2, levels=[(640, 1664), (128, 640), (0, 128)],
                          model_kwargs=dict(n_iters=ITERS, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                            ratio_threshold=None))
    pipe.run(batches)
    best = None
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = pipe.run(batches)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    C, H, W = 1664, 256, 256
    qps = nb * qb / best
    return {"queries_per_s": round(qps, 1), "roofline": pipeline_roofline(qps, None, robotcar=True),
            "ms_per_query": round(best / (nb * qb) * 1e3, 4),
            "batches": nb, "batch": qb, "points": N, "map": [C, H, W], "levels": [[640, 1664], [128, 640], [0, 128]],
            "statuses": sorted({r["status"] for b in res for r in b}),
            "pack_bytes_per_query": 8 * C * H * W,
            "note": "wall clock, host included; f-only pack (8C bytes per texel) + reference gather + 3 level "
                    "launches per batch, levels chained on the device"}


def pipeline_roofline(qps, window=None, root=ROOT, robotcar=False):
    """The end-to-end leg against the HBM roofline: the HBM bytes per query of its kernels (the
    f-only pack, the reference gather, the LM launches) from the committed rocprofv3 FETCH/WRITE
    summary of the same workload (profiles/rNN_pmc_pipeline.json, tools/gpu_profile_pipeline.sh),
    accepted only when taken with the loaded library's sources, times the wall-clock query rate."""
    from fmpnp import _lib
    digest = _lib.library_digest()
    why = []
    for rnd in PROFILE_ROUNDS:
        path = os.path.join("profiles", f"{rnd}_pmc_pipeline{'_w%d' % window if window else ''}"
                                        f"{'_robotcar' if robotcar else ''}.json")
        try:
            with open(os.path.join(root, path)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if digest == "unknown" or d.get("source_digest") != digest:
            why.append(f"{path}: taken with sources {d.get('source_digest')}, the loaded library is {digest}")
            continue
        if d.get("window") != window:
            why.append(f"{path}: window {d.get('window')}, the leg's is {window}")
            continue
        bpq = d["hbm_bytes_per_query"]
        ach = bpq * qps
        return {"bound": "hbm", "achieved": round(ach / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK, 4), "traffic": int(bpq),
                "traffic_unit": "HBM bytes per query (FETCH_SIZE x2 + WRITE_SIZE)", "source": path,
                "bytes_per_query_by_kernel": {k: int(v["hbm_bytes_per_query"]) for k, v in d["families"].items()},
                "kernel_us_per_query": round(d["kernel_ns_per_query"] / 1e3, 2),
                "kernel_bound_queries_per_s": round(1e9 / d["kernel_ns_per_query"], 1)}
    return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": None, "traffic": None,
            "source": "no committed PMC profile of this build (" + ("; ".join(why) or "none") + ")"}


def cpu_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return model, os.cpu_count(), affinity


def cpu_baseline(args, res_gpu, synth, dev):
    """CPU baselines on the GPU box's host, on queries the GPU refined in this run (global
    indices 0..S-1, S distinct maps): (1) the C restatement of the reference loop
    (oracle/fmpnp_oracle.c, OpenMP over queries) on every core of the job's CPU share;
    (2) the vectorised PyTorch-CPU fp64 restatement (oracle/ref_torch.py) at 1 thread and
    at that core count.  Both sides' poses are compared with the GPU's."""
    import oracle.oracle as orc
    from oracle import ref_torch
    model, ncpu, affinity = cpu_info()
    # the job's share of the host (OMP_NUM_THREADS: 16 per GPU on the pool's boxes)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity
    threads = args.cpu_threads or max(1, min(share, affinity))
    S = min(len(res_gpu), max(2 * threads, 16))
    maps = []
    for q in range(S):
        # the GPU run's own inputs (device generator), copied to the host in fp64 (exact)
        inp = synth.problem_inputs(N_PTS, C, HF, WF, seed=q, device=dev, init=args.init)
        fm = inp.pop("fmap").double().cpu().numpy()
        inp["fref"] = inp["fref"].double().cpu().numpy()
        gx, gy = orc.sobel(fm)
        maps.append((inp, fm, gx, gy))
    probs = [orc.make_problem(inp["pts3d"], inp["fref"], fm, gx, gy, inp["K"], inp["im_width"],
                              inp["im_height"], inp["R0"], inp["t0"]) for inp, fm, gx, gy in maps]
    copts = orc.make_options(ITERS, 0.01, "geman_mcclure", args.ratio)
    orc.lib()
    n_sample = max(S, args.cpu_sample)
    sample = [probs[i % S] for i in range(n_sample)]
    t = time.perf_counter()
    cres = orc.forward_batch(sample, copts, threads)
    dt = time.perf_counter() - t

    def cmp(poses):
        rot = max(rot_angle(p[0], g["R"]) for p, g in zip(poses, res_gpu))
        tr = max(float(np.linalg.norm(np.asarray(p[1]) - g["t"])) for p, g in zip(poses, res_gpu))
        return {"queries_compared": len(poses), "max_rot_diff_rad": rot, "max_t_diff_m": tr,
                "within_1e-4": bool(rot < 1e-4 and tr < 1e-4)}
    c_cmp = cmp([(r["R"], r["t"]) for r in cres[:S]])
    out = {"value": round(n_sample / dt, 4), "unit": "pose-refinements/s", "cores": threads, "kind": "port",
           "gn_iters_per_s": round(n_sample * ITERS / dt, 1),
           "sample": f"{n_sample} cfg2 problems = {S} distinct queries (global indices 0..{S - 1}, own map each) "
                     f"repeated, 50 iters, GM, fp64 CHW maps, C restatement, OpenMP {threads} threads, {dt:.1f}s",
           "cpu": model, "nproc": ncpu, "affinity_cpus": affinity, "job_cpu_share": share,
           "poses_vs_gpu": c_cmp}
    if not c_cmp["within_1e-4"]:
        log("[bench] WARNING: CPU (C oracle) and GPU poses differ by more than 1e-4", c_cmp)
    # the vectorised PyTorch-CPU fp64 restatement, 1 thread and the job's share
    tt = {}
    prev_threads = torch.get_num_threads()
    for nth, nq in ((1, 4), (threads, 2 * threads)):
        torch.set_num_threads(nth)
        nq = min(nq, S)
        poses = []
        t = time.perf_counter()
        for q in range(nq):
            inp, fm, gx, gy = maps[q]
            R, tv, _ = ref_torch.forward(inp["pts3d"], inp["fref"], fm, gx, gy, inp["K"], inp["im_width"],
                                         inp["im_height"], inp["R0"], inp["t0"], ITERS, 0.01, "geman_mcclure",
                                         args.ratio)
            poses.append((R.numpy(), tv.numpy()))
        dt = time.perf_counter() - t
        tt[f"threads_{nth}"] = {"value": round(nq / dt, 4), "unit": "pose-refinements/s", "cores": nth,
                                "sample": f"{nq} distinct cfg2 queries, 50 iters, {dt:.1f}s",
                                "poses_vs_gpu": cmp(poses)}
    torch.set_num_threads(prev_threads)
    out["pytorch_cpu_fp64"] = tt
    # (3) the library's CPU twin (fmpnp_refine_batch_cpu, include/fmpnp.h): the GPU's own packed fp32 maps
    # (the fp64 Sobel of the fp32 map rounded to fp32, as the pack kernel writes them), the LM kernel's
    # form of the loop on the same host threads -- a strong CPU baseline beside the reference-form port
    from fmpnp import _lib, cpu as fcpu, refine as rf
    St = min(S, max(threads, 4))
    hp = []
    for inp, fm, gx, gy in maps[:St]:
        feats = fcpu.pack_host(fm.astype(np.float32), gx.astype(np.float32), gy.astype(np.float32), np.float32)
        hp.append(fcpu.problem_host(feats, inp["fref"].astype(np.float32), inp["pts3d"], inp["K"], inp["im_width"],
                                    inp["im_height"], inp["R0"], inp["t0"]))
    topts = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, ratio_threshold=args.ratio, dtype=_lib.F32)
    n_twin = max(St, 16 * args.cpu_sample)
    t = time.perf_counter()
    tres, _ = fcpu.refine_cpu([hp[i % St] for i in range(n_twin)], topts, n_threads=threads)
    dt = time.perf_counter() - t
    out["cpu_twin"] = {"value": round(n_twin / dt, 2), "unit": "pose-refinements/s", "cores": threads,
                       "sample": f"{n_twin} cfg2 problems = {St} distinct queries repeated, 50 iters, GM, the packed "
                                 f"fp32 maps, fmpnp_refine_batch_cpu on {threads} threads, {dt:.1f}s",
                       "poses_vs_gpu": cmp([(r["R"], r["t"]) for r in tres[:St]])}
    del hp
    return out


if __name__ == "__main__":
    main()
