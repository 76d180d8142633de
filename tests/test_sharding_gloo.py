"""Multi-process (world_size 2, gloo, CPU) test of the query sharding used on N GPUs.

The compute of each shard here is the CPU oracle (test infrastructure) standing in
for the device refiner: this test covers the distribution plumbing -- contiguous
blocks, all-gather in global order, max-over-ranks timing -- not the kernel.  The
functions are the ones bench.py runs on N GPUs: fmpnp.shard.query_indices picks a
rank's queries (their global index seeds their inputs) and fmpnp.shard.timed_steps
brackets the timed launches.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fmpnp.shard import query_indices, shard_range


def test_shard_range_covers_all():
    for n in (0, 1, 7, 1024, 1025):
        for w in (1, 2, 3, 8):
            blocks = [shard_range(n, r, w) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            for (a, b), (c, d) in zip(blocks, blocks[1:]):
                assert b == c
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1


def test_query_indices_weak_and_strong():
    # weak scaling: B per rank, blocks of the global index space; strong: a fixed total split
    for world in (1, 2, 4, 8):
        weak = [list(query_indices(r, world, per_rank=128)) for r in range(world)]
        assert sum(weak, []) == list(range(128 * world))
        strong = [list(query_indices(r, world, global_batch=1024)) for r in range(world)]
        assert sum(strong, []) == list(range(1024))
        assert all(len(b) == 1024 // world for b in strong)
    # the rank-0 share of the weak form is the same queries at every world size
    assert list(query_indices(0, 8, per_rank=128)) == list(query_indices(0, 1, per_rank=128))


def _problem(i):
    import oracle.oracle as orc
    from golden_io import case, maps64
    names = ["gm_c16", "cauchy_c16", "odd_geom_gm", "behind_camera_gm", "huber_c16"]
    inp, meta, _ = case(names[i % len(names)])
    f, gx, gy = maps64(inp, orc.sobel)
    t0 = np.asarray(inp["t0"]) * (1.0 + 0.1 * i)
    return orc.make_problem(inp["pts3d"], inp["fref"], f, gx, gy, inp["K"], inp["im_width"], inp["im_height"],
                            inp["R0"], t0)


def _refine(probs):
    import oracle.oracle as orc
    opts = orc.make_options(8, 0.01, "geman_mcclure")
    return [dict(R=r["R"].tolist(), t=r["t"].tolist(), best_cost=r["best_cost"])
            for r in orc.forward_batch(probs, opts, 1)]


def _worker(rank, world, port, n, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "featuremetric-pnp_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import time
    from fmpnp.shard import max_over_ranks, query_indices, refine_sharded, timed_steps
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = refine_sharded(_problem, n, _refine)
    m = max_over_ranks(float(rank + 1))
    # bench.py's timed region: rank 1 is slower; every rank reports the slowest rank's time
    steps = []
    el = timed_steps(lambda k: (steps.append(k), time.sleep(0.05 * (rank + 1))), 3)
    mine = list(query_indices(rank, world, per_rank=3))
    got = [None] * world
    dist.all_gather_object(got, (el, steps, mine))
    if rank == 0:
        q.put((res, m, got))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(240)
def test_two_rank_gloo_matches_single_process():
    n = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res, m, got = q.get(timeout=200)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = _refine([_problem(i) for i in range(n)])
    assert m == 2.0
    (el0, st0, q0), (el1, st1, q1) = got
    assert el0 == el1 and el0 >= 0.3  # max over ranks: rank 1's 3 x 0.1 s
    assert st0 == st1 == [0, 1, 2]
    assert q0 == [0, 1, 2] and q1 == [3, 4, 5]
    assert len(res) == n
    for a, b in zip(res, single):
        assert a["R"] == b["R"] and a["t"] == b["t"] and a["best_cost"] == b["best_cost"]


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return r.returncode, lines, r.stderr


def test_bench_gpus_n_starts_n_ranks():
    """`python bench.py --gpus 2` (the driver's form, no launcher) starts two rank processes
    itself; each sees WORLD_SIZE 2 and takes its own block of queries (dry run: no GPU)."""
    rc, lines, err = _bench(["--gpus", "2", "--batch", "3"], {"FMPNP_BENCH_DRYRUN": "1", "FMPNP_BENCH_NDEV": "2"})
    assert rc == 0, err
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 for d in lines)
    assert sorted(d["device"] for d in lines) == [0, 1]
    assert all(d["n_gpus"] == 2 and d["ranks_per_device"] == 1.0 for d in lines)
    by_rank = {d["rank"]: d["queries"] for d in lines}
    assert by_rank[0] + by_rank[1] == list(range(6))


def test_bench_strong_form_splits_the_total():
    rc, lines, err = _bench(["--gpus", "2", "--global-batch", "5"], {"FMPNP_BENCH_DRYRUN": "1", "FMPNP_BENCH_NDEV": "2"})
    assert rc == 0, err
    by_rank = {d["rank"]: d["queries"] for d in lines}
    assert by_rank[0] + by_rank[1] == list(range(5))


def test_bench_refuses_a_rank_count_other_than_gpus():
    """Under a launcher, --gpus must equal WORLD_SIZE: never report an n_gpus other than the
    ranks that actually ran."""
    rc, lines, err = _bench(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "FMPNP_BENCH_DRYRUN": "1"})
    assert rc == 2 and not lines
    assert "WORLD_SIZE" in err


def test_bench_refuses_more_nccl_ranks_than_gpus():
    """One process per GPU: with the nccl backend, more ranks than visible GPUs is an error (the
    launcher used to map the surplus ranks onto one device silently and report them as GPUs)."""
    rc, lines, err = _bench(["--gpus", "2"], {"FMPNP_BENCH_DRYRUN": "1", "FMPNP_BENCH_NDEV": "1"})
    assert rc != 0 and not lines
    assert "visible GPU" in err


def test_bench_gloo_rehearsal_counts_one_gpu():
    """The gloo rehearsal (two ranks on a one-GPU box) reports n_gpus 1, ranks 2."""
    rc, lines, err = _bench(["--gpus", "2"], {"FMPNP_BENCH_DRYRUN": "1", "FMPNP_BENCH_NDEV": "1",
                                              "FMPNP_BENCH_BACKEND": "gloo"})
    assert rc == 0, err
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["n_gpus"] == 1 and d["ranks"] == 2 and d["ranks_per_device"] == 2.0 for d in lines)


def test_device_accounting():
    from fmpnp.shard import device_accounting
    assert device_accounting([("h", 0, 3, 0)]) == (1, 1.0)
    assert device_accounting([("h", 0, 3, 0), ("h", 0, 3, 0)]) == (1, 2.0)
    assert device_accounting([("h", 0, 3, 0), ("h", 0, 4, 0), ("h", 0, 5, 0), ("h", 0, 6, 0)]) == (4, 1.0)
    assert device_accounting([0, 1, 0, 1]) == (2, 2.0)


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_roofline_profile_must_match_kernel_and_build(tmp_path):
    """bench.py's roofline takes bytes from a committed PMC profile only when the profile names
    the kernel specialisation the launch ran AND was taken with the loaded library's sources;
    otherwise it reports why and falls back to live gathered bytes."""
    import json
    bench = _bench_module()
    (tmp_path / "profiles").mkdir()
    k6 = "fmpnp::lm_kernel<float, 2, false, false, 6>"

    def write(rnd, kernel, digest, nbytes=123):
        with open(tmp_path / "profiles" / f"{rnd}_pmc_b128_easy.json", "w") as f:
            json.dump({"kernel": f"void {kernel}(fmpnp::LaunchArgs)", "source_digest": digest,
                       "hbm_bytes_per_launch": nbytes, "kernel_avg_ns": 1000.0}, f)

    write("r03", k6, "aaaa", 100)
    got = bench.load_traffic("b128_easy", k6, "aaaa", root=str(tmp_path))
    assert got[0] == 100 and got[1] == k6 and got[4] is None
    # another build of the same kernel: rejected with the reason
    got = bench.load_traffic("b128_easy", k6, "bbbb", root=str(tmp_path))
    assert got[0] is None and "taken with sources aaaa" in got[4]
    # another specialisation (e.g. the ratio variant's profile under the plain tag): rejected
    got = bench.load_traffic("b128_easy", "fmpnp::lm_kernel<float, 2, false, true, 6>", "aaaa", root=str(tmp_path))
    assert got[0] is None and "is not the launch's" in got[4]
    # a newer round's profile of another build does not hide an older matching one
    write("r04", k6, "cccc", 200)
    got = bench.load_traffic("b128_easy", k6, "aaaa", root=str(tmp_path))
    assert got[0] == 100 and got[3].endswith("r03_pmc_b128_easy.json")
    # a library built outside the Makefile has no digest: never matched
    got = bench.load_traffic("b128_easy", k6, "unknown", root=str(tmp_path))
    assert got[0] is None
    # no profile at all
    got = bench.load_traffic("b999_easy", k6, "aaaa", root=str(tmp_path))
    assert got[0] is None and "no profiles" in got[4]


def test_pipeline_roofline_profile_must_match_build_and_window(tmp_path, monkeypatch):
    """The end-to-end leg's roofline takes bytes per query from a committed pipeline profile only
    when it was taken with the loaded library's sources and the leg's pack window."""
    import json
    bench = _bench_module()
    from fmpnp import _lib
    monkeypatch.setattr(_lib, "library_digest", lambda: "aaaa")
    (tmp_path / "profiles").mkdir()

    def write(name, digest, window, bpq):
        with open(tmp_path / "profiles" / name, "w") as f:
            json.dump({"source_digest": digest, "window": window, "hbm_bytes_per_query": bpq,
                       "kernel_ns_per_query": 20000.0, "families": {"pack": {"hbm_bytes_per_query": bpq}}}, f)

    write("r04_pmc_pipeline_w5.json", "aaaa", 5, 1e8)
    write("r04_pmc_pipeline.json", "aaaa", None, 2e8)
    got = bench.pipeline_roofline(30000.0, 5, root=str(tmp_path))
    assert got["traffic"] == 100000000 and got["frac"] == round(1e8 * 3e4 / bench.HBM_PEAK, 4)
    got = bench.pipeline_roofline(30000.0, None, root=str(tmp_path))
    assert got["traffic"] == 200000000 and got["source"].endswith("r04_pmc_pipeline.json")
    write("r04_pmc_pipeline_w5.json", "aaaa", 6, 1e8)  # another radius under the name: refused
    got = bench.pipeline_roofline(30000.0, 5, root=str(tmp_path))
    assert got["frac"] is None and "window 6" in got["source"]
    write("r04_pmc_pipeline_w5.json", "bbbb", 5, 1e8)  # another build: refused
    got = bench.pipeline_roofline(30000.0, 5, root=str(tmp_path))
    assert got["frac"] is None and "taken with sources bbbb" in got["source"]


def test_kernel_name_of_launch_plan():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "bid", os.path.join(ROOT, "featuremetric-pnp_amd", "fmpnp", "build_id.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.kernel_name(dict(dtype=0, build=2, team=0, ratio=0, variant=6)) == \
        "fmpnp::lm_kernel<float, 2, false, false, 6>"
    assert m.kernel_name(dict(dtype=1, build=4, team=1, ratio=1, variant=0)) == \
        "fmpnp::lm_kernel<double, 4, true, true, 0>"
    d = m.source_digest(ROOT)
    assert len(d) == 16 and d == m.source_digest(ROOT)
