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


def test_roofline_is_the_8d_byte_fraction_and_pmc_fractions_use_the_profiled_time(tmp_path, monkeypatch):
    """The line's roofline is SURVEY 8(d)'s: algorithmic bytes (nodes x 64 B + tests x 36 B + 32 B per
    pixel) over the live kernel time against 8 TB/s; every PMC fraction recomputes from the
    committed profile alone (its own launch time and clock), the live time does not enter them."""
    b = _bench()
    pt = SimpleNamespace(RayTracer=SimpleNamespace(KERNEL_TRIS=2))
    wl = "w"
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_roofline.json").write_text(json.dumps({wl: {
        "avg_kernel_ms_rocprof": 170.0, "hbm_bytes_per_launch": 2.0e10, "effective_clock_ghz": 2.2,
        "sq_insts_valu": 1.1e11, "sq_insts_salu": 4.3e10, "ta_busy_avr": 2.2e8, "valu_issue_frac": 0.55,
        "salu_issue_frac": 0.41, "ta_busy_frac": 0.33, "source": "x"}}))
    (prof / "gather_ceiling.json").write_text(json.dumps({"best_grec_per_s": 200.0, "source": "y"}))
    monkeypatch.setattr(b, "ROOT", tmp_path)
    cnt = {"nodes_visited": 18e9, "tris_tested": 6e9, "leaves_visited": 6e9, "lane_slots": 40e9}
    chain = {"alone_ms": 60.0, "pixel": [1, 2], "queries": 10, "steps": 100, "in_frame_ms": 150.0}
    pix = 1920 * 1080
    r = b.roofline_block(pt, 2, cnt, "bvh", pix, 160.0, wl, 1, chain, 1.1e9)
    fr = r["fractions"]
    assert set(fr) == {"hbm_pmc", "valu_issue", "salu_issue", "vmem_address", "record_gather", "critical_path"}
    assert all(0 < v["frac"] <= 1 for v in fr.values())
    alg = 18e9 * 64 + 6e9 * 36 + pix * 32
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - alg / 0.160 / 8e12) < 1e-4 and r["algorithmic_bytes_per_launch"] == int(alg)
    assert r["traffic"] == 2.0e10
    # the PMC fractions are the profile's own: live time 160 ms does not enter them
    assert fr["valu_issue"]["frac"] == 0.55 and fr["salu_issue"]["frac"] == 0.41
    assert abs(fr["hbm_pmc"]["frac"] - 2.0e10 / 0.170 / 8e12) < 1e-4
    assert abs(fr["critical_path"]["frac"] - 60.0 / 160.0) < 1e-4
    assert r["limiter"] == max(fr, key=lambda k: fr[k]["frac"])
    # another workload (or a tile) has no PMC entry: only the counter-based fractions remain
    r2 = b.roofline_block(pt, 2, cnt, "bvh", pix, 160.0, "other", 1, None, 1.1e9)
    assert set(r2["fractions"]) == {"record_gather"} and r2["traffic"] is None


def test_gpus_without_a_launcher_refuses_more_ranks_than_devices(monkeypatch):
    """bench.py --gpus N (no WORLD_SIZE): N ranks are started by bench.py itself; on a node with fewer
    GPUs than N (RCCL, one rank per GPU) it exits non-zero with a message instead of measuring one."""
    import subprocess

    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BENCH_DIST_BACKEND"] = "nccl"
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "GPU" in p.stderr and p.stdout == ""
