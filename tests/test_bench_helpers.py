"""bench.py's host-side helpers (CPU): the algorithmic FLOP count behind roofline.achieved, the
build-matched counter lookup behind roofline.traffic / issue, the parity summary, the core count."""
import json
import os

import numpy as np
import pytest


@pytest.fixture(scope="module")
def bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_bp_flops_per_sweep(bench):
    # 15 306 FP64 flops per message-passing sweep (ldpc_decoder.py:88-108)
    assert bench.bp_flops_per_pass() == 15306


def test_counters_for_build_matches_the_running_build(bench, tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    files = {"r2_v17_pmc.json": "B", "r3_v2_pmc.json": "A", "r3_v10_pmc.json": "B", "r3_v9_pmc.json": "C"}
    for name, bid in files.items():
        (prof / name).write_text(json.dumps({"build_id": bid, "kernels": {"k_bp": {"src": name}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    k, src = bench.counters_for_build("r*_v*_pmc.json", "B")
    assert src == os.path.join("profiles", "r3_v10_pmc.json") and k["k_bp"]["src"] == "r3_v10_pmc.json"
    k, src = bench.counters_for_build("r*_v*_pmc.json", "A")
    assert src == os.path.join("profiles", "r3_v2_pmc.json")
    k, src = bench.counters_for_build("r*_v*_pmc.json", "Z")   # no summary of this build: flagged stale
    assert k is None and src.startswith("stale: profiles/r3_v10_pmc.json (build B)")
    assert bench.counters_for_build("r*_v*_nothing.json", "B") == (None, None)


def test_parity_summary(bench):
    dt = np.dtype([("payload", "u1", (10,)), ("crc_calculated", "<u2"), ("abs_time", "<i4"),
                   ("abs_freq", "<i4"), ("score", "<f4")])
    g = np.zeros(2, dt)
    g["payload"][0, 0], g["payload"][1, 0] = 1, 2
    g["crc_calculated"] = [7, 9]
    g["abs_time"] = [960, 1920]
    g["abs_freq"] = [100, 200]
    g["score"] = [3.5, 4.0]
    cpu = [(bytes(r["payload"]).hex(), int(r["crc_calculated"]), int(r["abs_time"]) / 12000,
            (int(r["abs_freq"]) / 2) * 6.25, float(r["score"]) + 1e-6) for r in g]
    p = bench.parity_check([g], [cpu])
    assert p["payload_crc_multiset_equal"] and p["ordered_lists_equal_slots"] == 1
    assert 0 < p["max_abs_score_diff"] < 1e-5
    p = bench.parity_check([g], [cpu[:1]])
    assert p["mismatching_slots"] == [0] and p["decodes_gpu"] == 2 and p["decodes_cpu"] == 1


def test_host_cores(bench):
    n, basis = bench.host_cores()
    assert n >= 1 and "sched_getaffinity" in basis


def test_gather_check_and_shard_sample(bench):
    """The N > 1 line's self-check of the gathered decodes (bench.gather_check) and the per-rank
    sample lookup (bench.shard_sample) on a hand-made two-rank exchange."""
    from ft8_demodulator_amd._lib import RESULT_DTYPE
    S, world, cap = 3, 2, 4
    counts = np.array([[1, 0, 2, 0], [0, 3, 1, 0]])          # S_pad 4: one zero pad column
    slots = [0, 2, 2, 4, 4, 4, 5]
    flat = np.zeros(len(slots), RESULT_DTYPE)
    flat["slot"] = slots
    flat["payload"][:, 0] = np.arange(len(slots))
    ok = bench.gather_check(flat, counts, [3, 4], S, world, 7, cap)
    assert ok["gather_ok"] and ok["records"] == 7
    # a record under the wrong rank, a lost record, a wrong all-reduced count
    bad = flat.copy()
    bad["slot"][2] = 3
    assert not bench.gather_check(bad, counts, [3, 4], S, world, 7, cap)["gather_ok"]
    assert not bench.gather_check(flat[:-1], counts, [3, 3], S, world, 6, cap)["gather_ok"]
    assert not bench.gather_check(flat, counts, [3, 4], S, world, 8, cap)["gather_ok"]
    per = bench.shard_sample(flat, 3, 3)
    assert [len(p) for p in per] == [0, 3, 1]
    assert per[1]["payload"][:, 0].tolist() == [3, 4, 5]


def test_counters_for_build_takes_headline_passes_only(tmp_path, monkeypatch):
    """The headline line's traffic / issue counters come from r<round>_v<k>_pmc*.json of the running
    build -- never from a leg's summary of the same build (r4_v23_sub_pmc_traffic.json)."""
    import json
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    for name, bid in (("r4_v23_pmc_traffic.json", "B"), ("r4_v23_sub_pmc_traffic.json", "B"),
                      ("r4_v22_geo_pmc_traffic.json", "B"), ("r4_v19_pmc_traffic.json", "A")):
        (prof / name).write_text(json.dumps({"build_id": bid, "kernels": {"k": {"from": name}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    k, src = bench.counters_for_build("r*_pmc_traffic.json", "B")
    assert src == "profiles/r4_v23_pmc_traffic.json" and k["k"]["from"] == "r4_v23_pmc_traffic.json"
    k, src = bench.counters_for_build("r*_pmc_traffic.json", "C")
    assert k is None and src.startswith("stale: profiles/r4_v23_pmc_traffic.json")


def test_bp_cpu_baseline_threads(bench):
    """bench.bp_cpu_baseline (bp_stress's CPU leg): every sample vector decoded, rate and
    extrapolation reported with the thread count."""
    from oracle import oracle as O
    rng = np.random.default_rng(5)
    xn = np.stack([O.normalize(rng.standard_normal(174) * 2.0) for _ in range(24)])
    out = bench.bp_cpu_baseline(xn, 5, 3, 100000)
    assert out["cores"] == 3 and out["kind"] == "port" and out["value"] > 0
    assert out["extrapolated_s_per_launch"] == 100000 / out["value"]
    assert out["sample"].startswith("24 of")


def test_settle_stop_rule(bench):
    """The clock-settle phase stops on the first block within 1.5 % of the one before (the driver's
    --warmup 5 lines showed the first timed pairs ~10 % slower than the last)."""
    blocks = [33.0, 15.9, 15.0, 14.95]
    stops = [i for i in range(1, len(blocks)) if bench.settled(blocks[i - 1], blocks[i])]
    assert stops == [3]
    assert not bench.settled(None, 15.0)
    assert bench.settled(15.0, 15.2) and not bench.settled(15.0, 15.3)


def _fixture(name):
    root = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(root, "data", name)) as f:
        return json.load(f)


def _check_line(s, n_gpus):
    assert len(s.encode()) <= 4096, len(s.encode())
    assert "\n" not in s
    d = json.loads(s, parse_constant=lambda c: (_ for _ in ()).throw(ValueError(c)))   # strict: no NaN/Infinity
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "settle_steps", "ms_per_step", "config",
              "dtype", "roofline", "cpu_baseline", "parity", "depth", "build_id", "legs"):
        assert k in d, k
    assert d["n_gpus"] == n_gpus
    for k in ("kernel", "achieved", "peak", "frac", "launch_ms", "traffic", "traffic_source", "clock_effective_ghz"):
        assert k in d["roofline"], k
    return d


def test_compact_line_n1(bench):
    """The r05 line (23.8 KB, which the driver could not parse) -> one strict-JSON line <= 4 KB with
    the contract fields, roofline, cpu_baseline, a parity summary and the settle steps."""
    full = _fixture("bench_full_n1_r5.json")
    full["settle_steps"] = full["settle"]["steps"]
    full["roofline"]["frac"] = float("nan")      # a non-finite number must not leak into the line
    s = bench.compact_line(full, "gpurun_out/bench_legs.json")
    d = _check_line(s, 1)
    assert d["roofline"]["frac"] is None
    assert d["value"] == pytest.approx(full["value"], rel=1e-5)
    assert d["settle_steps"] == full["settle"]["steps"] and d["warmup"] == full["warmup"]
    for k in ("value", "unit", "cores", "kind"):
        assert d["cpu_baseline"][k] == pytest.approx(full["cpu_baseline"][k], rel=1e-5) \
            if isinstance(full["cpu_baseline"][k], float) else d["cpu_baseline"][k] == full["cpu_baseline"][k]
    assert d["parity"]["equal"] is True and d["parity"]["slots"] == full["parity"]["slots"]
    assert d["depth"]["one_chain_value"] == pytest.approx(full["depth"]["one_chain"]["value"], rel=1e-5)
    assert d["legs"] == "gpurun_out/bench_legs.json"


def test_compact_line_n8(bench):
    """A synthetic N = 8 record (the N = 4 rehearsal's, widened to 8 ranks with every per-rank array
    and the legs at their largest) still gives a line <= 4 KB carrying only the exchange's verdicts."""
    full = _fixture("bench_full_n4_r5.json")
    g = full["gather"]
    g["world"] = 8
    g["shard_parity"] = [dict(g["shard_parity"][0], rank=r, mismatching_slots=list(range(32)))
                         for r in range(8)]
    g["decodes_per_rank_last_step"] = [12345] * 8
    full["n_gpus"] = 8
    full["settle_steps"] = 96
    full["data"] = "x" * 3000                  # an over-long free-text field is shed, numbers stay
    s = bench.compact_line(full, "/tmp/legs.json")
    d = _check_line(s, 8)
    assert set(d["gather"]) == {"backend", "world", "gather_ok", "shard_parity_ok"}
    assert d["gather"]["world"] == 8 and d["settle_steps"] == 96


def test_write_legs_strict(bench, tmp_path):
    full = {"a": float("inf"), "b": [1.0, float("nan")], "c": np.float32(2.5), "d": np.int64(3)}
    p = bench.write_legs(full, str(tmp_path / "legs" / "x.json"))
    with open(p) as f:
        txt = f.read()
    assert json.loads(txt) == {"a": None, "b": [1.0, None], "c": 2.5, "d": 3}
