"""bench.py's profile selection (CPU): the roofline's traffic and executed-LU
figures come only from committed profiles stamped with the loaded library's
build id, newest by the timestamp recorded inside each file (not by name)."""
import json
import os

import bench


def _write(d, name, payload, jsonl=False):
    p = os.path.join(d, "profiles", name)
    with open(p, "w") as fh:
        if jsonl:
            fh.write("log line\n" + json.dumps(payload) + "\n")
        else:
            json.dump(payload, fh)


def test_selection_by_build_id_and_timestamp(tmp_path, monkeypatch):
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    k = bench.TRACK_KERNEL
    # a later-sorting name from another build must not win
    _write(tmp_path, "r9z_pmc_summary.json",
           {"build_id": "v0+other", "kernel": k, "measured_at": "2099", "derived": {"hbm_bytes_per_launch": 1}})
    _write(tmp_path, "r4aa_pmc_summary.json",
           {"build_id": "v1+abc", "kernel": k, "measured_at": "2026-10-17T10:00", "avg_ns": 2.5e7,
            "derived": {"hbm_bytes_per_launch": 7}})
    _write(tmp_path, "r4b_pmc_summary.json",
           {"build_id": "v1+abc", "kernel": k, "measured_at": "2026-10-17T09:00", "derived": {"hbm_bytes_per_launch": 5}})
    _write(tmp_path, "r4c_pmc_summary.json",   # same build, another kernel: skipped
           {"build_id": "v1+abc", "kernel": "other", "measured_at": "2027", "derived": {"hbm_bytes_per_launch": 3}})
    v, src = bench.traffic_bytes(k, "v1+abc")
    # the bytes come with the same profile's kernel time (the HBM rate's denominator)
    assert v == (7, 2.5e7) and src == os.path.join("profiles", "r4aa_pmc_summary.json")
    v, why = bench.traffic_bytes(k, "v1+none")
    assert v is None and "v1+none" in why


def test_lu_fraction_skips_scaled_runs(tmp_path, monkeypatch):
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    _write(tmp_path, "a_lu_work.json", {"build_id": "b", "measured_at": "2", "config": "config 2 scaled x10",
                                        "executed_fraction": 0.9}, jsonl=True)
    _write(tmp_path, "b_lu_work.json", {"build_id": "b", "measured_at": "1", "config": "config 2",
                                        "executed_fraction": 0.42}, jsonl=True)
    v, src = bench.lu_executed_fraction("b")
    assert v == 0.42 and src.endswith("b_lu_work.json")


def test_wilson_interval():
    """Config 5's success-rate interval (bench.wilson95): Wilson 95 % score interval."""
    lo, hi = bench.wilson95(6, 10)
    assert abs(lo - 0.3127) < 1e-3 and abs(hi - 0.8318) < 1e-3
    assert bench.wilson95(0, 30)[0] == 0.0 and bench.wilson95(30, 30)[1] == 1.0
    assert bench.wilson95(0, 0) is None


def test_committed_bench_line_keeps_the_contract():
    """The shipped build's committed bench line (profiles/r7i_bench.json) carries
    every field of the driver's contract, a roofline and CPU baseline of the
    right shape, the HBM traffic of its own build, and small launches faster
    on the latency-mode kernel than on the throughput one."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = json.load(open(os.path.join(root, "profiles", "r7i_bench.json")))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "f32"
    assert abs(d["value"] - 31200 / (d["ms_per_step"] / 1e3)) / d["value"] < 1e-3
    assert "config 2" in d["config"]["workload"]
    r = d["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(r)
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3 and 0 < r["frac"] < 1
    assert r["traffic_source"] == "profiles/r7i_pmc_summary.json"
    c = d["cpu_baseline"]
    assert {"value", "unit", "cores", "kind", "sample"} <= set(c) and c["kind"] in ("port", "reference")
    s = d["config"]["small_launch"]
    assert s["samples"] == [1, 8]
    assert all(a < b for a, b in zip(s["latency_kernel_ms"], s["throughput_kernel_ms"]))
    assert d["config"]["build_id"] == json.load(open(os.path.join(root, r["traffic_source"])))["build_id"]
