"""bench.py's host-side helpers (no GPU): the committed PMC profile it quotes, and the CPU leg's
per-channel RMSE check (oracle restatement vs an image) on a small case."""
import numpy as np

import bench
import minimal_volumetric_path_tracer_amd as vpt
from oracle.oracle import Oracle


def test_pmc_profile_only_for_its_build(tmp_path, monkeypatch):
    """a PMC profile is quoted only by the library build it was collected on (profiles/r*/pmc_*.json
    carry build_id, scripts/pmc_summary.py); newest round first"""
    import json
    import os

    base = json.load(open(os.path.join(bench.ROOT, "profiles", "r03", "pmc_pool_kernel.json")))
    for rnd, bid in (("r98", "aaaa"), ("r99", "bbbb")):
        os.makedirs(tmp_path / "profiles" / rnd)
        json.dump(dict(base, build_id=bid), open(tmp_path / "profiles" / rnd / "pmc_pool_kernel.json", "w"))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    p = bench.pmc_profile("ff", 1, "aaaa")
    assert p is not None and p["build_id"] == "aaaa" and p["path"] == os.path.join("profiles", "r98", "pmc_pool_kernel.json")
    assert bench.pmc_profile("ff", 1, "cccc") is None
    assert bench.pmc_profile("mis", 1, "aaaa") is None and bench.pmc_profile("ff", 2, "aaaa") is None
    t = bench.pmc_traffic(p)
    assert t == int((2 * p["counters"]["FETCH_SIZE"] + p["counters"]["WRITE_SIZE"]) * 1024) and t > 0
    assert bench.pmc_fp64_flop(p) > 0
    c = bench.CONFIGS["ff"]
    f = bench.pmc_fields(p, 50.0, bench.fb_bytes(c), bench.partial_bytes(c))
    assert abs(f["hbm_gbs"] - t / 0.05 / 1e9) < 0.01 and 0 < f["valu_busy"] < 1 and 0 < f["lane_util"] < 1
    assert bench.fb_bytes(c) == 1024 * 1024 * 12 and bench.partial_bytes(c) == 1024 * 1024 * 24 * 16
    assert f["traffic_over_partials"] == round(t / bench.partial_bytes(c), 3) and f["pmc_build_id"] == "aaaa"
    assert all(v is None for v in bench.pmc_fields(None, 50.0, 1, 1).values())


def test_partial_bytes_match_the_chunk_layout():
    """bench's partial byte count uses the auto layout of csrc/vpt_chunks.h (via the C library's plan)"""
    import test_launch_plan as tlp

    for cfg in bench.CONFIGS.values():
        units, _ = tlp.units_of(cfg["width"], cfg["height"], cfg["spp"])
        tiles = ((cfg["width"] + 7) // 8) * ((cfg["height"] + 7) // 8) * 64
        assert bench.partial_bytes(cfg) == cfg["width"] * cfg["height"] * 24 * (units // tiles)


def test_cpu_port_check_rmse():
    c = dict(width=48, height=32, spp=3, estimator="ff", sigma_a=0.001, sigma_s=0.009)
    o = Oracle(portable=True)
    o.set_scene(vpt.default_scene())
    img = o.render(48, 32, 3, 0, seed=0x5EED0001, threads=2).astype(np.float32)
    r = bench.cpu_port_check(img, c, threads=2, bands=2, band=16, cal_spp=1)
    assert r["kind"] == "port" and r["rmse_vs_gpu_per_channel"] == [0.0, 0.0, 0.0] and r["value"] > 0
    img[0, 5, 1] += 0.5  # file row 0 = camera row 31, inside the top band
    assert bench.cpu_port_check(img, c, threads=2, bands=2, band=16, cal_spp=1)["rmse_vs_gpu_per_channel"][1] > 0


def test_bench_configs_match_baseline():
    assert bench.CONFIGS["ff"] == dict(width=1024, height=1024, spp=256, estimator="ff", sigma_a=0.001, sigma_s=0.009)
    assert bench.CONFIGS["mis4k"]["spp"] == 8192 and bench.CONFIGS["mis4k"]["width"] == 4096


def test_reference_estimator_rate_multiprocess():
    """the north-star CPU leg: the reference's MIS estimator in one process per core (oracle/ref_rate.py)"""
    import os
    import pytest
    from oracle.oracle import Reference

    if not Reference.available():
        pytest.skip("oracle/_ref/libvpt_ref.so not built")
    cpus = sorted(os.sched_getaffinity(0))[:2]
    c = dict(width=32, height=16, spp=4, estimator="mis", sigma_a=0.001, sigma_s=0.009)
    r = bench.reference_estimator_rate(1, c, cpus, rows_per=2, spp=4)
    assert r["cores"] == len(cpus) and r["value"] > 0
    assert f"{len(cpus)} processes" in r["sample"]


def test_socket_conservative_uses_the_fastest_runs():
    """the conservative socket figure (the denominator of the quoted GPU/CPU ratios) takes the fastest run
    of each set, so a slow outlier lowers the ratio, never raises it; and it is never below one core x 64"""
    # 16-core runs 18, 20, 22 Msamples/s; one-core 1.1, 1.3, 1.2
    assert bench.socket_conservative([18.0, 20.0, 22.0], [1.1, 1.3, 1.2], 16, 64) == max(22.0 * 4, 1.3 * 64)
    # poor 16-core scaling: the one-core figure decides
    assert bench.socket_conservative([12.0, 13.0, 11.0], [1.3, 1.25, 1.2], 16, 64) == 1.3 * 64
    # a slowed run cannot raise the ratio: adding a slower run leaves the figure unchanged
    assert bench.socket_conservative([22.0, 10.0], [1.3, 0.5], 16, 64) == bench.socket_conservative([22.0], [1.3], 16, 64)


def test_shared_device_refusal():
    """an N-GPU bench line needs N distinct GPUs (PCI ids) unless --shared-device marks a test run"""
    assert bench.shared_device_refusal(["0000:05:00", "0000:15:00"], False) is None
    assert bench.shared_device_refusal(["0000:05:00"], False) is None
    why = bench.shared_device_refusal(["0000:05:00", "0000:15:00", "0000:05:00"], False)
    assert why and "0000:05:00" in why and "3-GPU" in why
    assert bench.shared_device_refusal(["0000:05:00", "0000:05:00"], True) is None
