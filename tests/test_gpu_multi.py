"""GPU tests of the node-level entry points: vpt_render_multi / vpt_multi_* (include/vpt.h; several
GPUs of one process, strips gathered over RCCL) and the `vpt` program, the drop-in for the
reference's `./rt <spp>` (src/rt.cpp:744-830: image.ppm in the reference's format and the
"elapsed time: <s>s" line of src/rt.cpp:824-827).

The box these run on has one GPU: the multi-GPU entry is exercised with n_gpus = 1, and its n > 1 path
with n logical ranks sharing device 0 (vpt_debug_multi_create_shared: everything but the RCCL send /
recv, which becomes a same-device copy); the gloo tests of test_distributed.py cover the Python path's
band layout, and the 8-GPU run is the driver's."""
import dataclasses
import os
import re
import subprocess

import numpy as np
import pytest
from conftest import bitwise_equal

import minimal_volumetric_path_tracer_amd as vpt

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VPT = os.path.join(ROOT, "minimal_volumetric_path_tracer_amd", "vpt")


@pytest.mark.parametrize("est,fp64", [("ff", True), ("mis", True), ("ff", False)])
def test_multi_one_gpu_equals_render(gpu_tracer, est, fp64):
    gpu_tracer.set_scene(vpt.default_scene())
    cfg = vpt.RenderConfig(width=48, height=40, spp=3, estimator=est, fp64=fp64, seed=31)
    ref = gpu_tracer.render(cfg)
    m = vpt.MultiTracer(1)
    try:
        a = m.render(cfg)
        b = m.render(cfg)  # the handle's buffers are reused
    finally:
        m.close()
    assert bitwise_equal(a, ref).all() and bitwise_equal(b, ref).all()
    assert bitwise_equal(vpt.render_multi(1, cfg), ref).all()


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("est,fp64,h,band", [("ff", True, 40, 0), ("mis", True, 37, 0), ("ff", False, 53, 4),
                                             ("mis", False, 16, 0)])
def test_multi_shared_device_n_ranks_equals_render(gpu_tracer, n, est, fp64, h, band):
    """vpt_multi_render's n > 1 path executed on the one-GPU box: n logical ranks
    on device 0 (vpt_debug_multi_create_shared), each with its context, stream and strip, its bands
    rendered on its own stream, the strips moved into device 0's gather buffer by stream-ordered copies
    where RCCL's grouped send / recv would run, then the band plan's device-to-host copies.  Bit-identical
    to vpt_render for ragged heights (bands that do not divide the image, ranks with no band at all:
    n = 8 over 16 rows), both framebuffer formats and two calls on the same handle (buffers reused)."""
    gpu_tracer.set_scene(vpt.default_scene())
    cfg = vpt.RenderConfig(width=24, height=h, spp=3, estimator=est, fp64=fp64, seed=29,
                           band_rows=band if band else 0)
    ref = gpu_tracer.render(dataclasses.replace(cfg, band_rows=0))
    m = vpt.MultiTracer(n, shared_device=True)
    try:
        a = m.render(cfg)
        b = m.render(dataclasses.replace(cfg, seed=29))
    finally:
        m.close()
    assert bitwise_equal(a, ref).all() and bitwise_equal(b, ref).all()


def test_multi_band_rows_argument(gpu_tracer):
    """a caller band size that cuts the image is accepted (the layout does not change the bits)"""
    gpu_tracer.set_scene(vpt.default_scene())
    cfg = vpt.RenderConfig(width=32, height=36, spp=2, fp64=True, seed=5)
    ref = gpu_tracer.render(cfg)
    import dataclasses

    got = vpt.render_multi(1, dataclasses.replace(cfg, band_rows=8))
    assert bitwise_equal(got, ref).all()


def test_multi_invalid_arguments():
    import torch

    ndev = torch.cuda.device_count()
    with pytest.raises(vpt.VPTError):
        vpt.MultiTracer(ndev + 1)
    with pytest.raises(vpt.VPTError):
        vpt.MultiTracer(0)
    with pytest.raises(vpt.VPTError):  # a shard, not the whole image
        vpt.render_multi(1, vpt.RenderConfig(width=8, height=32, spp=1, band_rows=8, band_stride=2, band_offset=1))


def _run_vpt(args, cwd):
    r = subprocess.run([VPT] + [str(a) for a in args], cwd=cwd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout


@pytest.mark.parametrize("extra,est", [([], 0), (["--estimator", "mis"], 1), (["--gpus", "1"], 0)])
def test_cli_ppm_equals_oracle(orc_vm, tmp_path, extra, est):
    """`vpt 4 --width 64 --height 48 --seed 7 --fp64`: the bytes of the oracle's render written by
    the reference's PPM writer (restated in the oracle, src/rt.cpp:812-820), and the reference's
    timing line"""
    out = _run_vpt([4, "--width", 64, "--height", 48, "--seed", 7, "--fp64", "--out", "x.ppm"] + extra, tmp_path)
    assert re.fullmatch(r"elapsed time: [0-9.e+-]+s\n", out), out
    orc_vm.set_scene(vpt.default_scene())  # the CLI renders the reference scene
    lin = orc_vm.render(64, 48, 4, est, seed=7)
    orc_vm.write_ppm(str(tmp_path / "o.ppm"), lin)
    assert (tmp_path / "x.ppm").read_bytes() == (tmp_path / "o.ppm").read_bytes()


def test_cli_default_float32_framebuffer(orc_vm, tmp_path):
    """without --fp64 the framebuffer is float32 (vpt_params.fb_format): the PPM is the writer applied
    to the float32 averages"""
    _run_vpt([2, "--width", 40, "--height", 30, "--seed", 9], tmp_path)
    orc_vm.set_scene(vpt.default_scene())
    lin = orc_vm.render(40, 30, 2, 0, seed=9).astype(np.float32)
    orc_vm.write_ppm(str(tmp_path / "o.ppm"), lin)
    assert (tmp_path / "image.ppm").read_bytes() == (tmp_path / "o.ppm").read_bytes()


@pytest.mark.parametrize("prog", ["rt_vpt", "rt_vpt_multi"])
def test_integration_dropin_program_runs(tmp_path, prog):
    """INTEGRATION.md section 1 executed: the reference's own main() (src/rt.cpp) with the drop-in
    blocks in place of its pixel loop and PPM writer, built by __graft_entry__.build() from a copy of
    the reference sources (oracle/dropin.py).  `rt_vpt 2` renders the reference's 1024x768 image at
    2 spp through vpt_render (rt_vpt_multi: vpt_render_multi over every GPU present), prints the
    reference's timing line and writes image.ppm -- byte-identical to the library's own render of
    the same default parameters encoded by the PPM writer."""
    exe = os.path.join(ROOT, "oracle", "_ref", prog)
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built (needs the reference checkout at build time)")
    r = subprocess.run([exe, "2"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert re.search(r"elapsed time: [0-9.e+-]+s", r.stdout), r.stdout[-500:]
    t = vpt.Tracer(0)
    try:
        img = t.render(vpt.RenderConfig(width=1024, height=768, spp=2))
    finally:
        t.close()
    assert (tmp_path / "image.ppm").read_bytes() == vpt.encode_ppm(img)


def test_cli_rejects_bad_arguments(tmp_path):
    for args in (["x"], ["0"], ["4", "--estimator", "nope"], ["4", "--gpus", "0"], ["4", "--width"]):
        r = subprocess.run([VPT] + args, cwd=tmp_path, capture_output=True, text=True, timeout=60)
        assert r.returncode == 2 and "usage" in r.stderr, args
