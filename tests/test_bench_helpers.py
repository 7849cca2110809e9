"""bench.py's host-side helpers (no GPU): the committed PMC profile it quotes, and the CPU leg's
per-channel RMSE check (oracle restatement vs an image) on a small case."""
import numpy as np

import bench
import minimal_volumetric_path_tracer_amd as vpt
from oracle.oracle import Oracle


def test_committed_pmc_profile_is_read():
    p = bench.pmc_profile("ff", 1)
    assert p is not None and "pool_kernel<0, false>" in p["dispatch"]["kernel"]
    t = bench.pmc_traffic(p)
    assert t == int((2 * p["counters"]["FETCH_SIZE"] + p["counters"]["WRITE_SIZE"]) * 1024) and t > 0
    assert bench.pmc_fp64_flop(p) > 0
    assert bench.pmc_profile("mis", 1) is None and bench.pmc_profile("ff", 2) is None


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
