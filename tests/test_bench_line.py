"""bench.py's stdout line stays small enough for the driver to parse it whole (round 4's 20.5 KB
line was cut to its last 8 KB and left unparsed): the headline keys plus one summary per leg,
every leg's full record in a side file referenced by path and sha256."""
import hashlib
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_line_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _canned():
    # the full round-4 default line (every leg, 20.5 KB) as the canned result set
    with open(os.path.join(ROOT, "profiles", "r04_bench_default.json")) as f:
        return json.load(f)


def test_compact_line_fits_and_keeps_the_headline(tmp_path):
    bench = _bench()
    full = _canned()
    full["facade_call"] = {"cfg2": {"ms_per_call": 1.234, "calls_per_s": 810.4},
                           "robotcar_n295": {"ms_per_call": 2.5, "calls_per_s": 400.0}}
    ref = bench.write_detail(full, str(tmp_path / "d" / "bench_detail.json"))
    line = bench.compact_line(full, ref)
    text = json.dumps(line)
    assert len(text) <= bench.LINE_MAX_BYTES, len(text)
    assert len(text) <= 12000
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "gn_iters_per_s", "statuses"):
        assert k in line, k
    assert line["value"] == full["value"] and line["metric"] == full["metric"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert "legs_dropped" not in line
    legs = line["legs"]
    for k in ("single_query", "hard_init", "hard_init_ratio08", "ratio08", "layout_f", "end_to_end",
              "end_to_end.full_pack", "end_to_end.robotcar_1664", "pyramid_robotcar_1664",
              "pyramid_robotcar_1664.median_query_n295", "fixed_total_1024", "no_memo", "pack",
              "facade_call.cfg2", "facade_call.robotcar_n295"):
        assert k in legs, k
        assert "ms" in legs[k] or "rate" in legs[k], (k, legs[k])
    assert legs["hard_init"]["frac"] == full["hard_init"]["roofline"]["frac"]
    assert legs["facade_call.cfg2"]["ms"] == 1.234
    # the side file is what the line names
    with open(ref["path"], "rb") as f:
        blob = f.read()
    assert hashlib.sha256(blob).hexdigest() == ref["sha256"] and len(blob) == ref["bytes"]
    assert json.loads(blob)["pyramid_robotcar_1664"] == full["pyramid_robotcar_1664"]


def test_compact_line_drops_legs_before_the_headline():
    bench = _bench()
    full = _canned()
    for i in range(400):  # far more legs than fit
        full[f"extra_leg_{i}"] = {"ms_per_launch": 1.0, "pose_refinements_per_s": 2.0, "roofline": {"frac": 0.5}}
    line = bench.compact_line(full, {"path": None})
    assert len(json.dumps(line)) <= bench.LINE_MAX_BYTES
    assert line["legs_dropped"] > 0 and line["roofline"]["frac"] == full["roofline"]["frac"]
    assert "cpu_baseline" in line and "single_query" in line["legs"]
