"""bench.py host logic (no GPU): CPU accounting and the roofline's fraction bookkeeping."""
from __future__ import annotations

import importlib.util
import json
import sys
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["bench_mod"] = mod
    spec.loader.exec_module(mod)
    return mod


def test_host_cpus_reports_threads_within_affinity():
    b = _bench()
    hc = b.host_cpus()
    assert 1 <= hc["threads"] <= hc["affinity"] <= (hc["nproc"] or hc["affinity"])
    if hc["cgroup_quota_cpus"]:
        assert hc["threads"] <= hc["cgroup_quota_cpus"]


def test_roofline_bound_is_the_largest_fraction(tmp_path, monkeypatch):
    b = _bench()
    pt = SimpleNamespace(RayTracer=SimpleNamespace(KERNEL_TRIS=2))
    wl = "w"
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_roofline.json").write_text(json.dumps({wl: {
        "hbm_bytes_per_launch": 2.0e10, "effective_clock_ghz": 2.4, "sq_insts_valu": 1.1e11,
        "sq_insts_salu": 4.3e10, "ta_busy_avr": 2.2e8, "source": "x"}}))
    (prof / "gather_ceiling.json").write_text(json.dumps({"best_grec_per_s": 200.0, "source": "y"}))
    monkeypatch.setattr(b, "ROOT", tmp_path)
    cnt = {"nodes_visited": 18e9, "tris_tested": 6e9, "leaves_visited": 6e9, "lane_slots": 40e9}
    chain = {"alone_ms": 60.0, "pixel": [1, 2], "queries": 10, "steps": 100, "in_frame_ms": 150.0}
    r = b.roofline_block(pt, 2, cnt, "bvh", 1920 * 1080, 160.0, wl, 1, chain, 1.1e9)
    fr = r["fractions"]
    assert set(fr) == {"hbm", "valu_issue", "salu_issue", "vmem_address", "record_gather", "critical_path"}
    assert all(0 < v["frac"] <= 1 for v in fr.values()) and r["fractions_over_1"] == []
    assert r["bound"] == max(fr, key=lambda k: fr[k]["frac"])
    assert r["frac"] == fr[r["bound"]]["frac"]
    assert abs(fr["valu_issue"]["frac"] - 1.1e11 / 0.16 / 1e9 / (1024 * 2.4 / 2)) < 1e-3
    assert abs(fr["critical_path"]["frac"] - 60.0 / 160.0) < 1e-4
    # another workload (or a tile) has no PMC entry: only the counter-based fractions remain
    r2 = b.roofline_block(pt, 2, cnt, "bvh", 1920 * 1080, 160.0, "other", 1, None, 1.1e9)
    assert set(r2["fractions"]) == {"record_gather"} and r2["traffic"] is None
