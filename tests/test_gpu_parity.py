"""GPU parity: libvpt.so's HIP kernels against the oracle and the reference's fixtures.

Bars (Parity):
  * bit-exact vs the oracle's portable-math build (oracle/liboracle_vm.so) -- every per-sample
    value, every random-stream end state, every framebuffer value, every math-library result;
  * vs the reference's own outputs (tests/golden/, glibc libm): identical random-draw trajectories
    and green/blue channels within 1e-9 relative for >= 99 % of samples; the red channel differs
    only through the reference's rounding-coin-flip hazards, checked statistically.
"""
import ctypes
import os

import numpy as np
import pytest
from conftest import GOLDEN, bitwise_equal
from scenes import SCENES

import minimal_volumetric_path_tracer_amd as vpt
from minimal_volumetric_path_tracer_amd import _lib

pytestmark = pytest.mark.gpu
SEED = 0x5EED0001


def _rays(r6):
    r = np.zeros(len(r6), dtype=vpt.RAY_DTYPE)
    r["o"], r["d"] = r6[:, :3], r6[:, 3:]
    return r


# ---------------------------------------------------------------- math library
@pytest.mark.parametrize("fn,lo,hi", [
    (0, 0, 1e6), (1, -745, 710), (2, 1e-300, 1e300), (3, -7, 7), (4, -7, 7), (5, -1.5, 1.5), (6, -1e3, 1e3),
    (7, -1, 1), (8, -100, 100), (9, -1e3, 1e3), (10, -1, 1), (11, -1, 1)])
def test_device_math_bitwise(gpu_tracer, orc, orc_vm, fn, lo, hi):
    rng = np.random.default_rng(fn)
    x = rng.uniform(lo, hi, 200000)
    y = rng.uniform(-100, 100, 200000)
    if fn == 2:
        x = np.exp(rng.uniform(-690, 690, 200000))
    special = np.array([0.0, -0.0, 1.0, -1.0, 0.5, -0.5, np.pi, np.pi / 2, 1e-310, np.inf, -np.inf, np.nan])
    x = np.concatenate([x, special])
    y = np.concatenate([y, special[::-1]])
    dev = gpu_tracer.math_probe(fn, x, y)
    # the device's lm_* == the oracle's portable build == glibc itself (orc: libm build and,
    # parametrized, the portable one)
    for host in (orc_vm.math(fn, x, y), orc.math(fn, x, y)):
        same = bitwise_equal(dev, host)
        assert same.all(), f"fn {fn}: {(~same).sum()} differ, e.g. x={x[~same][:3]} dev={dev[~same][:3]} host={host[~same][:3]}"


def test_device_dir_trig_cone_path_vs_glibc(gpu_tracer):
    """the cone samplers' trig (lm_dir_trig with every lane's c > 0.9925: gm_sincos_acos_phi_cone, where
    cos(acos c) is taken to be c -- VPT_COS_ACOS_C, csrc/vpt_glibm.h) against glibc's own sin(acos c),
    cos(acos c), sin(phi), cos(phi) bit for bit: 4 M uniform c in (0.9925, 1], the 2^17 doubles just below 1,
    c = 1, and the range's low end"""
    from oracle.oracle import Oracle

    glibc = Oracle(portable=False)
    rng = np.random.default_rng(2606)
    n = 1 << 22
    top = 1.0 - np.arange(0, 1 << 17) * 2.0**-53
    low = np.nextafter(0.9925, 1.0) + np.arange(0, 4096) * 2.0**-53
    c = np.concatenate([rng.uniform(0.9925, 1.0, n), top, low])
    c = np.maximum(c, np.nextafter(0.9925, 1.0))
    c = np.concatenate([c, np.full(64 - len(c) % 64, 1.0)])  # whole waves of cone-range lanes
    phi = 2 * np.pi * rng.random(len(c))
    for fn in (14, 15, 16, 17):
        dev = gpu_tracer.math_probe(fn, c, phi)
        ref = glibc.math(fn, c, phi)
        same = bitwise_equal(dev, ref)
        assert same.all(), f"fn {fn}: {(~same).sum()} differ, e.g. c={c[~same][:3]}"
    assert bitwise_equal(gpu_tracer.math_probe(15, c, phi), c).all()  # cos(acos c) == c there


def test_device_isect_sqrt_tiny(gpu_tracer):
    """VPT_ISECT_CLASS / VPT_ISECT_ZERO (csrc/vpt_math.h vm_sqrt_isect, vm_sqrt_isect_z): the sphere tests' root equals sqrt() bit for bit for
    det = 0, inf, NaN, negative and every det >= 2^-767, and for det in (0, 2^-767) -- subnormals included,
    where it runs the core sequence -- is a finite number below 2^-383, the bound the sphere test's
    exactness argument needs (sq below half an ulp of any |b| >= 2^-330)"""
    rng = np.random.default_rng(2703)
    n = 1 << 20
    big = np.ldexp(rng.uniform(1, 2, n), rng.integers(-767, 1024, n))
    edge = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, -1.0, 2.0**-767, np.nextafter(2.0**-767, 0),
                     1.7976931348623157e308])
    x = np.concatenate([big, edge, np.tile(edge, 64)])
    with np.errstate(invalid="ignore"):
        ref = np.sqrt(x)
    sel = ~((x > 0) & (x < 2.0**-767))
    assert bitwise_equal(gpu_tracer.math_probe(21, x)[sel], ref[sel]).all()
    # every binade below 2^-767 (normal and subnormal), whole waves of them
    e = rng.integers(-1074, -767, n)
    tiny = np.ldexp(rng.uniform(1, 2, n), e)
    tiny = np.concatenate([tiny, np.array([5e-324, 1e-320, 2.0**-1022, np.nextafter(2.0**-1022, 0)])])
    r = gpu_tracer.math_probe(21, tiny)
    assert np.isfinite(r).all() and (r >= 0).all() and (r < 2.0**-383).all()
    # the shadow rays' root (VPT_ISECT_ZERO, vm_sqrt_isect_z): zeros join the tiny range (a finite root below
    # 2^-383 instead of the rare-argument call), everything else as above
    with np.errstate(invalid="ignore"):
        assert bitwise_equal(gpu_tracer.math_probe(22, x)[sel & (x != 0)], ref[sel & (x != 0)]).all()
    z = np.concatenate([tiny, np.zeros(4096), -np.zeros(4096)])
    r = gpu_tracer.math_probe(22, z)
    assert np.isfinite(r).all() and (r >= 0).all() and (r < 2.0**-383).all()


def test_device_shared_reciprocal_division(gpu_tracer):
    """VPT_DIV_SHARE (csrc/vpt_math.h vm_rcp, csrc/vpt_device.h): the last three operations of the
    compiler's division on a reciprocal formed once per divisor give the division's bits for operands in
    [2^-300, 2^300); hemiCosineProb's c / pi on the constant RN(1/pi), and the 1 / d, r / d pairs of the
    cone samplers, equal the divisions everywhere (their range tests send the rest to the plain division)"""
    rng = np.random.default_rng(2608)
    n = 1 << 21
    a = np.ldexp(rng.uniform(1, 2, n), rng.integers(-300, 299, n)) * rng.choice([-1.0, 1.0], n)
    b = np.ldexp(rng.uniform(1, 2, n), rng.integers(-300, 299, n)) * rng.choice([-1.0, 1.0], n)
    b[: n // 4] = rng.uniform(0.5, 400, n // 4)  # the path's divisors: distances, 2 pi (1 - c), ...
    a[: n // 8] = 1.0
    assert bitwise_equal(gpu_tracer.math_probe(18, a, b), a / b).all()
    assert bitwise_equal(gpu_tracer.math_probe(18, a, np.full(n, np.pi)), a / np.pi).all()
    edge = np.array([0.0, -0.0, 5e-324, -5e-324, 1e-310, 2.0**-300, np.nextafter(2.0**-300, 0), 2.0**300,
                     np.nextafter(2.0**300, 0), 1e300, np.inf, -np.inf, np.nan, 1.0, -1.0])
    c = np.concatenate([rng.uniform(-1, 1, n), edge, np.tile(edge, 64)])  # whole waves of edge values too
    with np.errstate(all="ignore"):
        assert bitwise_equal(gpu_tracer.math_probe(19, c), c * 1 / np.pi).all()
    d = np.concatenate([rng.uniform(1e-3, 500, n), edge, np.tile(edge, 64)])
    r = rng.choice([0.0, 2.0, 16.5, 1e5, -0.0], len(d))
    r[-len(edge):] = edge[::-1]
    with np.errstate(all="ignore"):
        want = (1 / d).view(np.uint64) ^ (r / d).view(np.uint64)
    got = gpu_tracer.math_probe(20, d, r).view(np.uint64)
    assert np.array_equal(got, want), f"{(got != want).sum()} differ"


def test_device_atan2_wide_and_range_bounds(gpu_tracer, orc):
    """gm_atan2 on the device (its two divisions by max(|y|, x) on one reciprocal, VPT_DIV_SHARE; operands
    outside [2^-300, 2^300] to the translated library) against glibc over every exponent of both operands
    and around the 2^-300 / 2^300 bounds, bit for bit"""
    from oracle.oracle import Oracle

    glibc = Oracle(portable=False)
    rng = np.random.default_rng(2609)
    n = 1 << 20
    x = np.ldexp(rng.uniform(1, 2, n), rng.integers(-1000, 1000, n))
    y = np.ldexp(rng.uniform(1, 2, n), rng.integers(-1000, 1000, n)) * rng.choice([-1.0, 1.0], n)
    b = np.array([2.0**-300, np.nextafter(2.0**-300, 0), np.nextafter(2.0**-300, 1), 2.0**300,
                  np.nextafter(2.0**300, 0), np.nextafter(2.0**300, np.inf), 1.0, 3.0, 1e-10, 1e10])
    bx, by = np.meshgrid(b, np.concatenate([b, -b]))
    x = np.concatenate([x, bx.ravel(), rng.uniform(0, 300, n)])
    y = np.concatenate([y, by.ravel(), rng.uniform(-400, 400, n)])
    dev = gpu_tracer.math_probe(8, y, x)
    ref = glibc.math(8, y, x)
    same = bitwise_equal(dev, ref)
    assert same.all(), f"{(~same).sum()} differ, e.g. y={y[~same][:3]} x={x[~same][:3]}"


def test_device_tan_range_boundaries(gpu_tracer, orc):
    """gm_tan on the device over the ranges the [-1.5, 1.5] sweep above leaves out: [1.5,
    pi/2) -- the odd-n branch where -1/y goes through the double-double division, reached by the
    equi-angular sampler's tan near +-pi/2 -- and (0.787, 25] after the reduction by pi/2; plus the CPU
    test's range bounds and table-node boundaries (tests/test_glibc_libm.py::test_tan_range_boundaries),
    against glibc's tan bit for bit"""
    rng = np.random.default_rng(306)
    nodes = (np.arange(0, 190) + 15.5) / 256
    bounds = np.array([float.fromhex(h) for h in ("0x1.b096cp-27", "0x1.f212dp-5", "0x1.92f1ap-1")] + [25.0])
    x = np.concatenate([nodes, np.pi / 2 - nodes, np.pi / 2 + nodes, bounds, np.nextafter(bounds, 0),
                        np.nextafter(bounds, 1), np.pi / 4 * np.arange(-31, 32), rng.uniform(1.5, np.pi / 2, 100_000),
                        np.pi / 2 - np.exp(rng.uniform(-40, -3, 20_000)), rng.uniform(0.787, 25.0, 100_000)])
    x = np.concatenate([x, -x])
    got, want = gpu_tracer.math_probe(5, x), orc.math(5, x)
    same = bitwise_equal(got, want)
    assert same.all(), f"{(~same).sum()} of {len(x)} differ, e.g. x={x[~same][:4]}"


@pytest.mark.parametrize("est", ["ff", "mis", "explicit_free", "explicit"])
def test_kill_prediction_draw_counts(gpu_tracer, est):
    """the pool's kill-predicting rings (vpt_pool.h) assume a diffuse surface event draws 2 n_mis + 4
    samples and a medium event 4 before the next roulette draw; vpt_count_work's counting kernel checks
    that on every event it traces and fails (VPT_E_INTERNAL) otherwise -- over the test and
    alternate scenes, with HG and a depth cap"""
    from scenes import ALT_SCENES, EST_SCENES

    for name, mk in list(EST_SCENES.items()) + list(ALT_SCENES.items()):
        gpu_tracer.set_scene(mk())
        for kw in ({}, dict(hg_g=0.5), dict(max_depth=3)):
            tests, iters = gpu_tracer.count_work(vpt.RenderConfig(width=24, height=16, spp=8, estimator=est, **kw))
            assert tests > 0 and iters > 0, (name, kw)
    gpu_tracer.set_scene(vpt.default_scene())


def _debug_fn(name, argtypes):
    f = getattr(vpt.lib(), name)
    f.restype = ctypes.c_int
    f.argtypes = argtypes
    return f


@pytest.mark.parametrize("est", ["ff", "mis"])
def test_kill_prediction_check_can_fail(gpu_tracer, est):
    """the draw-count check above must be able to fail: with the kill prediction's surface
    jump one draw off (vpt_debug_kill_jump: 2 n_mis + 6 instead of 2 n_mis + 5 draws to the roulette),
    vpt_count_work raises VPT_E_INTERNAL; with the scene's own jump restored it passes again"""
    jump = _debug_fn("vpt_debug_kill_jump", [ctypes.c_void_p, ctypes.c_int])
    sc = vpt.default_scene()
    gpu_tracer.set_scene(sc)
    n_mis = int(((sc["r"] > 0) & (sc["radiance"][:, 0] > 0)).sum())
    cfg = vpt.RenderConfig(width=24, height=16, spp=8, estimator=est)
    _lib.check(jump(gpu_tracer._ctx, 2 * n_mis + 6))
    try:
        with pytest.raises(vpt.VPTError, match="kill prediction"):
            gpu_tracer.count_work(cfg)
    finally:
        _lib.check(jump(gpu_tracer._ctx, 0))
    tests, iters = gpu_tracer.count_work(cfg)
    assert tests > 0 and iters > 0


def test_karg_guard_fails_loudly(gpu_tracer):
    """pool_kernel reads its launch parameters from the kernel-argument segment at use (VPT_P_KARG); its
    layout guard, made to fail by vpt_debug_karg_guard, must not hand back a garbage image with VPT_OK
    (ADVICE r05): vpt_render returns VPT_E_INTERNAL, the device path's image is NaN, and with the hook
    cleared the render is the oracle's again"""
    guard = _debug_fn("vpt_debug_karg_guard", [ctypes.c_void_p, ctypes.c_uint])
    gpu_tracer.set_scene(vpt.default_scene())
    cfg = vpt.RenderConfig(width=16, height=16, spp=4, fp64=True, seed=SEED)
    good = gpu_tracer.render(cfg)
    _lib.check(guard(gpu_tracer._ctx, 1))
    try:
        with pytest.raises(vpt.VPTError, match="VPT_P_KARG"):
            gpu_tracer.render(cfg)
        import torch
        buf = torch.zeros((16, 16, 3), dtype=torch.float64, device="cuda:0")
        gpu_tracer.render_device(cfg, buf.data_ptr(), 0)
        torch.cuda.synchronize()
        assert torch.isnan(buf).all()
    finally:
        _lib.check(guard(gpu_tracer._ctx, 0))
    again = gpu_tracer.render(cfg)
    assert bitwise_equal(again, good).all() and np.isfinite(good).all()


def test_device_sqrt_div_correctly_rounded(gpu_tracer, orc):
    rng = np.random.default_rng(5)
    x = np.abs(rng.normal(size=300000)) * 10.0 ** rng.integers(-300, 300, 300000)
    y = rng.normal(size=300000) * 10.0 ** rng.integers(-300, 300, 300000)
    assert bitwise_equal(gpu_tracer.math_probe(0, x), np.sqrt(x)).all()
    assert bitwise_equal(gpu_tracer.math_probe(9, x, y), x / y).all()


def test_device_atan2_huge_ratio(gpu_tracer, orc):
    """gm_atan2's |y|/x > 2^57 shortcut (+-hpi; the equi-angular atan2(MAXFLOAT - proj, D) of an
    escaping ray) == glibc's atan2 on the device too"""
    rng = np.random.default_rng(13)
    x = np.exp(rng.uniform(-30, 30, 100000))
    y = x * 2.0 ** rng.uniform(50, 75, 100000) * rng.choice([-1.0, 1.0], 100000)
    D = np.exp(rng.uniform(-8, 7, 4000))
    ym = np.float64(3.4028234663852886e38) - rng.uniform(-400, 400, 4000)
    y, x = np.concatenate([y, ym, -ym]), np.concatenate([x, D, D])
    got, want = gpu_tracer.math_probe(8, y, x), orc.math(8, y, x)
    assert bitwise_equal(got, want).all()


def test_device_inv_sqrt_exact(gpu_tracer):
    """vm_inv_sqrt (nrm's 1.0 / sqrt(|a|^2): the square root and the division sequences without their
    scaling / fix-up steps inside [2^-767, DBL_MAX]) == 1.0 / np.sqrt(x) bit for bit, across the
    exponent range, at the fast path's ends, on exact squares and their neighbours, and on specials"""
    rng = np.random.default_rng(12)
    x = np.abs(rng.normal(size=400000)) * 10.0 ** rng.integers(-320, 309, 400000)
    lo = 2.0 ** -767
    edges = np.array([lo, np.nextafter(lo, 0), np.nextafter(lo, 1), 2.0 ** -1022, 5e-324, 1e-310,
                      np.finfo(np.float64).max, np.nextafter(np.finfo(np.float64).max, 0), 0.0, -0.0, -1.0,
                      np.inf, -np.inf, np.nan, 1.0, 4.0, 0.25, 2.0, 0.5])
    sq = (rng.integers(1, 1 << 26, 20000).astype(np.float64)) ** 2 * 2.0 ** rng.integers(-600, 600, 20000)
    near = np.concatenate([sq, np.nextafter(sq, 0), np.nextafter(sq, np.inf)])
    unit = 1.0 + rng.uniform(-1e-6, 1e-6, 100000)  # |a|^2 of nearly unit vectors (the path's common case)
    # roots s with an all-ones significand (the reciprocal's exceptional case): x around (2 - 2^-52)^2 2^(2k)
    ones = (2.0 - 2.0**-52) ** 2 * 4.0 ** rng.integers(-380, 500, 4000).astype(np.float64)
    ones = np.concatenate([ones, np.nextafter(ones, 0), np.nextafter(ones, np.inf), np.nextafter(np.nextafter(ones, 0), 0)])
    wide = np.ldexp(rng.uniform(1.0, 4.0, 2_000_000), 2 * rng.integers(-383, 511, 2_000_000))  # every exponent of [2^-767, DBL_MAX]
    x = np.concatenate([x, edges, near, unit, ones, wide])
    with np.errstate(divide="ignore", invalid="ignore"):
        want = 1.0 / np.sqrt(x)
    got = gpu_tracer.math_probe(12, x)
    same = bitwise_equal(got, want)
    assert same.all(), f"{(~same).sum()} differ, e.g. x={x[~same][:3]} got={got[~same][:3]} want={want[~same][:3]}"


def test_device_sqrt_edges(gpu_tracer):
    """vm_sqrt's unwrapped fast path covers [2^-767, DBL_MAX]; everything else (and the range
    ends) must give sqrt()'s bits too: zeros, subnormals, the 2^-767 boundary, inf, NaN,
    negatives, exact squares and their neighbours."""
    rng = np.random.default_rng(11)
    b = 2.0 ** -767
    edge = [0.0, -0.0, 5e-324, 2.2250738585072014e-308, np.nextafter(b, 0), b, np.nextafter(b, 1),
            1.7976931348623157e308, np.inf, -np.inf, np.nan, -1.0, -5e-324, 1.0, 4.0, 2.0]
    sq = rng.uniform(1, 2 ** 26, 20000).round() ** 2
    near = np.concatenate([sq, np.nextafter(sq, 0), np.nextafter(sq, np.inf)])
    tiny = rng.uniform(0.5, 2, 20000) * 2.0 ** rng.integers(-1074, -700, 20000)
    big = rng.uniform(0.5, 2, 20000) * 2.0 ** rng.integers(900, 1024, 20000)
    x = np.concatenate([edge, near, tiny, big, -tiny])
    with np.errstate(invalid="ignore", over="ignore"):
        ref = np.sqrt(x)
    dev = gpu_tracer.math_probe(0, x)
    same = (dev.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(dev) & np.isnan(ref))  # signed zeros too
    assert same.all(), f"{(~same).sum()} differ, e.g. x={x[~same][:3]}"



# ---------------------------------------------------------------- per-sample estimator
@pytest.fixture(scope="module")
def samples():
    return dict(np.load(os.path.join(GOLDEN, "samples.npz")))


@pytest.mark.parametrize("scene", list(SCENES))
@pytest.mark.parametrize("est", [0, 1])
def test_trace_batch_vs_oracle_bitwise(gpu_tracer, orc_vm, samples, scene, est):
    sc = samples[f"{scene}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    k = f"{scene}__e{est}__"
    rays, st = samples[k + "ray"], samples[k + "state1"]
    L, s = gpu_tracer.trace(est, _rays(rays), st)
    Lo, so = orc_vm.trace(est, rays, st)
    assert np.array_equal(s, so)
    same = bitwise_equal(L, Lo)
    assert same.all(), f"{(~same.all(1)).sum()} of {len(L)} samples differ"


@pytest.mark.parametrize("scene", list(SCENES))
@pytest.mark.parametrize("est", [0, 1])
def test_trace_batch_vs_reference(gpu_tracer, samples, scene, est):
    """against the reference's own per-sample values (its functions compiled here with glibc):
    the same random draws for every sample; free flight bit for bit, MIS within 1e-12 relative
    (the reference sums its recursion back to front) -- the device libm is glibc's
    (csrc/vpt_glibc.h), so no rounding-coin flip is re-rolled."""
    sc = samples[f"{scene}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    k = f"{scene}__e{est}__"
    L, s = gpu_tracer.trace(est, _rays(samples[k + "ray"]), samples[k + "state1"])
    ref = samples[k + "L"]
    assert np.array_equal(s, samples[k + "state2"]), "random draws consumed differ"
    if est == 0:
        same = bitwise_equal(L, ref)
        assert same.all(), f"{(~same.all(1)).sum()} of {len(L)} samples differ"
    else:
        close = bitwise_equal(L, ref) | (np.abs(L - ref) <= 1e-12 * np.maximum(np.abs(ref), 1e-300))
        assert close.mean() >= 0.999 and close.all(), f"{(~close.all(1)).sum()} of {len(L)} samples differ"


# ---------------------------------------------------------------- renders
@pytest.mark.parametrize("est", ["ff", "mis"])
def test_render_vs_oracle_bitwise(gpu_tracer, orc_vm, est):
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    e = 0 if est == "ff" else 1
    g64 = gpu_tracer.render(width=40, height=28, spp=3, estimator=est, seed=SEED, fp64=True)
    o = orc_vm.render(40, 28, 3, e, seed=SEED)
    assert bitwise_equal(g64, o).all()
    g32 = gpu_tracer.render(width=40, height=28, spp=3, estimator=est, seed=SEED)
    assert bitwise_equal(g32, o.astype(np.float32)).all()


@pytest.mark.parametrize("spp,chunk", [(40, 0), (40, 7), (40, 40), (40, 1), (33, 0), (70, 0)])
def test_chunked_sums_vs_oracle(gpu_tracer, orc_vm, spp, chunk):
    """samples summed in chunks (vpt_params.chunk_spp; auto = chunks of min(spp, 32), the last 32 tapered,
    csrc/vpt_chunks.h); chunk 1 or spp = reference order."""
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    g = gpu_tracer.render(width=20, height=12, spp=spp, chunk_spp=chunk, seed=4, fp64=True)
    eff = chunk if chunk > 0 else None  # None: the auto (tapered) layout
    o = orc_vm.render(20, 12, spp, 0, seed=4, chunk=eff, threads=4)
    assert bitwise_equal(g, o).all()
    if chunk in (1, spp):
        assert bitwise_equal(g, orc_vm.render(20, 12, spp, 0, seed=4, chunk=spp, threads=4)).all()


@pytest.mark.parametrize("g,depth", [(0.5, 0), (-0.3, 0), (0.0, 8), (0.7, 3)])
@pytest.mark.parametrize("est", [0, 1])
def test_extensions_vs_oracle(gpu_tracer, orc_vm, g, depth, est):
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    gp = gpu_tracer.render(width=24, height=16, spp=4, estimator=est, hg_g=g, max_depth=depth, sigma_a=0.01,
                           sigma_s=0.09, seed=3, fp64=True)
    o = orc_vm.render(24, 16, 4, est, hg_g=g, max_depth=depth, sigma_a=0.01, sigma_s=0.09, seed=3)
    assert bitwise_equal(gp, o).all()


def test_render_vs_reference_fixture(gpu_tracer):
    """vs the reference's own 64x64x16 renders (tests/golden/fb64x64x16_e*.npy): north_star's
    per-channel RMSE < 1e-4 on all three channels; in fact free flight is bit-identical and MIS
    differs by summation order only."""
    gpu_tracer.set_scene(SCENES["default"]())
    for est in (0, 1):
        ref = np.load(os.path.join(GOLDEN, f"fb64x64x16_e{est}.npy"))
        g = gpu_tracer.render(width=64, height=64, spp=16, estimator=est, seed=SEED + 1, fp64=True)
        assert np.isfinite(g).all()
        rmse = np.sqrt(((g - ref) ** 2).reshape(-1, 3).mean(0))
        assert (rmse < 1e-4).all(), (est, rmse)
        if est == 0:
            assert bitwise_equal(g, ref).all()
        else:
            np.testing.assert_allclose(g, ref, rtol=1e-12, atol=1e-300)
        g32 = gpu_tracer.render(width=64, height=64, spp=16, estimator=est, seed=SEED + 1)
        rmse32 = np.sqrt(((g32 - ref) ** 2).reshape(-1, 3).mean(0))
        assert (rmse32 < 1e-4).all(), (est, rmse32)


def test_shards_compose_bitwise(gpu_tracer):
    gpu_tracer.set_scene(SCENES["default"]())
    base = dict(width=32, height=40, spp=2, seed=11)
    full = gpu_tracer.render(**base)
    for bands, world in [(8, 2), (5, 3), (40, 1), (16, 4), (3, 5)]:
        parts = [gpu_tracer.render(**base, band_rows=bands, band_stride=world, band_offset=r) for r in range(world)]
        img = np.zeros_like(full)
        for r, part in enumerate(parts):
            rows = [fr for b in range(r, (40 + bands - 1) // bands, world) for fr in range(b * bands, min(40, (b + 1) * bands))]
            assert len(rows) == len(part)
            img[rows] = part
        assert np.array_equal(img, full)


def test_deterministic_and_seeded(gpu_tracer):
    gpu_tracer.set_scene(SCENES["default"]())
    a = gpu_tracer.render(width=64, height=48, spp=4, seed=5)
    b = gpu_tracer.render(width=64, height=48, spp=4, seed=5)
    c = gpu_tracer.render(width=64, height=48, spp=4, seed=6)
    assert np.array_equal(a, b) and not np.array_equal(a, c)


def test_overlapping_renders_on_one_context(gpu_tracer):
    """vpt_render_device is asynchronous: renders enqueued on several streams of ONE context are in
    flight together (each stream gets its own work queue and partials, vpt_kernels.hip
    stream_slot), and two renders queued back to back on one stream reuse its slot in order.  Every
    image equals the same render done alone.  Device buffers and streams come from the HIP runtime
    libvpt.so links (torch's wheel carries its own runtime, a second instance in the process)."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so.7")
    ok = lambda rc: rc == 0 or pytest.fail(f"HIP error {rc}")  # noqa: E731
    gpu_tracer.set_scene(SCENES["default"]())
    cfgs = [vpt.RenderConfig(width=64, height=48, spp=8, seed=21),
            vpt.RenderConfig(width=96, height=64, spp=12, estimator="mis", hg_g=0.5, seed=22),
            vpt.RenderConfig(width=32, height=32, spp=40, seed=23)]
    alone = [gpu_tracer.render(c) for c in cfgs]
    streams = [ctypes.c_void_p() for _ in range(2)]
    bufs = [ctypes.c_void_p() for _ in cfgs]
    for st in streams:
        ok(hip.hipStreamCreate(ctypes.byref(st)))
    try:
        for c, b in zip(cfgs, bufs):
            n = c.height * c.width * 3 * 4
            ok(hip.hipMalloc(ctypes.byref(b), ctypes.c_size_t(n)))
            ok(hip.hipMemset(b, 0xFF, ctypes.c_size_t(n)))  # NaN until written
        ok(hip.hipDeviceSynchronize())
        for i, (c, b) in enumerate(zip(cfgs, bufs)):  # renders 0 and 2 share stream 0, render 1 runs on stream 1
            gpu_tracer.render_device(c, b.value, streams[i % 2].value)
        ok(hip.hipDeviceSynchronize())
        for a, c, b in zip(alone, cfgs, bufs):
            got = np.empty((c.height, c.width, 3), dtype=np.float32)
            ok(hip.hipMemcpy(got.ctypes.data_as(ctypes.c_void_p), b, ctypes.c_size_t(got.nbytes), 2))  # device to host
            assert np.array_equal(a, got)
    finally:
        for b in bufs:
            if b.value:
                hip.hipFree(b)
        for st in streams:
            if st.value:
                hip.hipStreamDestroy(st)


def test_threads_and_many_streams_on_one_context(gpu_tracer):
    """Several host threads render on different streams of ONE context at once (the context's slot
    table is taken under its lock until the launches are enqueued; slots have stable addresses), and
    more streams than the table holds (8) take over finished slots: every image equals the same render
    done alone."""
    import ctypes
    import threading

    hip = ctypes.CDLL("libamdhip64.so.7")
    ok = lambda rc: rc == 0 or pytest.fail(f"HIP error {rc}")  # noqa: E731
    gpu_tracer.set_scene(SCENES["default"]())
    cfgs = [vpt.RenderConfig(width=48 + 8 * i, height=32, spp=6 + i, seed=100 + i, estimator="mis" if i % 3 == 0 else "ff")
            for i in range(12)]
    alone = [gpu_tracer.render(c) for c in cfgs]
    streams = [ctypes.c_void_p() for _ in cfgs]  # 12 streams > the 8 slots of a context
    bufs = [ctypes.c_void_p() for _ in cfgs]
    errors = []
    try:
        for st in streams:
            ok(hip.hipStreamCreate(ctypes.byref(st)))
        for c, b in zip(cfgs, bufs):
            n = c.height * c.width * 3 * 4
            ok(hip.hipMalloc(ctypes.byref(b), ctypes.c_size_t(n)))
            ok(hip.hipMemset(b, 0xFF, ctypes.c_size_t(n)))
        ok(hip.hipDeviceSynchronize())

        def worker(k):
            try:
                for i in range(k, len(cfgs), 4):
                    for _ in range(2):  # twice on its stream: the slot is reused in stream order
                        gpu_tracer.render_device(cfgs[i], bufs[i].value, streams[i].value)
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
        ok(hip.hipDeviceSynchronize())
        for a, c, b in zip(alone, cfgs, bufs):
            got = np.empty((c.height, c.width, 3), dtype=np.float32)
            ok(hip.hipMemcpy(got.ctypes.data_as(ctypes.c_void_p), b, ctypes.c_size_t(got.nbytes), 2))
            assert np.array_equal(a, got)
    finally:
        hip.hipDeviceSynchronize()
        for b in bufs:
            if b.value:
                hip.hipFree(b)
        for st in streams:
            if st.value:
                hip.hipStreamDestroy(st)


def test_band_shards_reassemble_like_multi_render(gpu_tracer):
    """The n > 1 data path of vpt_multi_render without RCCL: n "devices" render their interleaved
    row bands (band_stride n, band_offset g) into compact strips, the strips are packed into
    n slots as the RCCL gather leaves them on device 0, and the library's own reassembly
    (vpt_debug_band_reorder, the code vpt_multi_render runs) gives the whole image byte for byte."""
    import ctypes

    L = vpt.lib()
    L.vpt_debug_band_reorder.restype = ctypes.c_int
    L.vpt_debug_band_reorder.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_size_t, ctypes.c_void_p]
    gpu_tracer.set_scene(SCENES["default"]())
    for n, band, (w, h) in ((2, 16, (64, 96)), (3, 16, (40, 70)), (8, 16, (32, 200)), (8, 5, (24, 53))):
        whole = gpu_tracer.render(width=w, height=h, spp=4, seed=31)
        strips = [gpu_tracer.render(width=w, height=h, spp=4, seed=31, band_rows=band, band_stride=n, band_offset=g)
                  for g in range(n)]
        row_bytes = w * 3 * 4
        cap = max(len(s) for s in strips)
        staging = np.zeros((n, cap, w, 3), dtype=np.float32)
        for g, st in enumerate(strips):
            staging[g, :len(st)] = st
        out = np.full((h, w, 3), np.nan, dtype=np.float32)
        rc = L.vpt_debug_band_reorder(staging.ctypes.data, cap * row_bytes, n, h, band, row_bytes, out.ctypes.data)
        assert rc == 0
        assert out.tobytes() == whole.tobytes(), (n, band)


def test_count_work_matches_oracle(gpu_tracer, orc_vm):
    for name in ("default", "mat3", "dielectric"):
        sc = SCENES[name]()
        gpu_tracer.set_scene(sc)
        orc_vm.set_scene(sc)
        for est in (0, 1):
            t, it = gpu_tracer.count_work(vpt.RenderConfig(width=32, height=24, spp=4, estimator=est, seed=9))
            _, c = orc_vm.render(32, 24, 4, est, seed=9, counters=True)
            assert (t, it) == (c.tests, c.iterations)


def test_edge_cases(gpu_tracer, orc_vm):
    # 1x1 image, spp 1; no emitters; >4 emitters (the reference's arr[4] overflow is an extension here)
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    assert bitwise_equal(gpu_tracer.render(width=1, height=1, spp=1, fp64=True), orc_vm.render(1, 1, 1)).all()
    ne = SCENES["no_emitter"]()
    gpu_tracer.set_scene(ne)
    assert not gpu_tracer.render(width=8, height=8, spp=2).any()
    many = np.concatenate([sc] + [vpt.Sphere(1.0, (x, 30.0, -20.0), radiance=(20, 20, 20)) for x in (-30, -10, 10, 30)])
    gpu_tracer.set_scene(many)
    orc_vm.set_scene(many)
    assert bitwise_equal(gpu_tracer.render(width=16, height=12, spp=2, fp64=True, seed=2), orc_vm.render(16, 12, 2, seed=2)).all()
    gpu_tracer.set_scene(sc)


def test_invalid_arguments_raise(gpu_tracer):
    with pytest.raises(vpt.VPTError):
        gpu_tracer.render(width=0, height=4, spp=1)
    with pytest.raises(vpt.VPTError):
        gpu_tracer.render(width=4, height=4, spp=0)
    with pytest.raises(vpt.VPTError):
        gpu_tracer.render(width=4, height=4, spp=1, hg_g=1.0)
    with pytest.raises(vpt.VPTError):
        gpu_tracer.render(width=4, height=4, spp=1, band_rows=2, band_stride=2, band_offset=2)
    bad = SCENES["default"]()
    bad[3]["material"] = 7
    with pytest.raises(vpt.VPTError):
        gpu_tracer.set_scene(bad)
    with pytest.raises(vpt.VPTError):
        gpu_tracer.set_scene(np.concatenate([SCENES["default"]()] * 7))
    gpu_tracer.set_scene(SCENES["default"]())


def test_full_size_properties(gpu_tracer, orc_vm):
    """BASELINE configs[1] geometry (1024x1024) at 8 spp: deterministic, finite, a random set of
    pixels recomputed by the oracle bit for bit, image means near the reference's."""
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    img = gpu_tracer.render(width=1024, height=1024, spp=8, seed=SEED, fp64=True)
    assert np.isfinite(img).all()
    rng = np.random.default_rng(0)
    for fr in rng.integers(0, 1024, 6):
        y = 1023 - int(fr)
        row = orc_vm.render(1024, 1024, 8, 0, seed=SEED, y0=y, y1=y + 1)[fr]
        assert bitwise_equal(img[fr], row).all()
    # same camera geometry at 128x128x16 (independent samples) from the oracle: means agree within
    # 6 standard errors (per-sample sigma ~1.2)
    small = orc_vm.render(128, 128, 16, 0, seed=SEED + 99, threads=8)
    m, ms = img.reshape(-1, 3).mean(0), small.reshape(-1, 3).mean(0)
    se = np.sqrt(img.reshape(-1, 3).var(0) * 8 / img.size * 3 + small.reshape(-1, 3).var(0) * 16 / small.size * 3)
    assert np.all(np.abs(m - ms) <= 6 * se + 1e-6), (m, ms, se)


@pytest.mark.gpu
def test_config1_full_size_256spp_vs_oracle(gpu_tracer, orc_vm):
    """BASELINE configs[1] at its own size: FF 1024x1024x256 -- the bench workload -- with the auto
    chunk layout (6 x 32 samples, then the tapered 22, 14, 10, 6, 4, 3, 2, 1, 1, 1: 16 chunks,
    vpt_chunks.h), which only this sample count exercises at full size.  Six file rows, spread over
    the image, are recomputed by the oracle (the reference's pixel loop, src/rt.cpp:784-800, with the
    same per-sample streams and chunked sums) bit for bit; the whole image is finite."""
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    img = gpu_tracer.render(width=1024, height=1024, spp=256, seed=SEED, fp64=True)
    assert img.shape == (1024, 1024, 3) and np.isfinite(img).all()
    for fr in (0, 211, 512, 767, 901, 1023):
        y = 1023 - fr
        row = orc_vm.render(1024, 1024, 256, 0, seed=SEED, y0=y, y1=y + 1, threads=8)[fr]
        assert bitwise_equal(img[fr], row).all(), fr
    assert img.max() > 0


@pytest.mark.gpu
def test_config2_full_size_mis_hg_1024spp_vs_oracle(gpu_tracer, orc_vm):
    """BASELINE configs[2] -- the north-star workload -- at its own size: MIS (free flight +
    equi-angular, MISVPTTracerRecursive, include/vptShadeMethods.h:1345-1481) with HG g = 0.5,
    1024 x 1024 x 1024 spp, the auto layout at 1024 spp (30 x 32 samples, then the 64-sample taper:
    40 chunks), the pool at full occupancy.  Six file rows are recomputed by the oracle's pixel loop
    (src/rt.cpp:784-800, ~6 M CPU samples) bit for bit; the whole image is finite."""
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    img = gpu_tracer.render(width=1024, height=1024, spp=1024, estimator="mis", hg_g=0.5, seed=SEED, fp64=True)
    assert img.shape == (1024, 1024, 3) and np.isfinite(img).all() and img.max() > 0
    for fr in (0, 187, 511, 640, 888, 1023):
        y = 1023 - fr
        row = orc_vm.render(1024, 1024, 1024, 1, hg_g=0.5, seed=SEED, y0=y, y1=y + 1, threads=16)[fr]
        assert bitwise_equal(img[fr], row).all(), fr


@pytest.mark.gpu
def test_config3_full_size_dense_depth8_4096spp_vs_oracle(gpu_tracer, orc_vm):
    """BASELINE configs[3] at its own size: free flight in the dense medium (sigma_t 0.03), paths capped
    at 8 vertices, 2048 x 2048 x 4096 spp (126 x 32-sample chunks + the taper: 136 chunks, 13.7 GB
    of partials).  Two file rows (~17 M CPU samples) recomputed by the oracle bit for bit; the whole
    image is finite and lit."""
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    kw = dict(sigma_a=0.003, sigma_s=0.027, max_depth=8)
    img = gpu_tracer.render(width=2048, height=2048, spp=4096, estimator="ff", seed=SEED, fp64=True, **kw)
    assert img.shape == (2048, 2048, 3) and np.isfinite(img).all() and img.max() > 0
    for fr in (5, 1400):
        y = 2047 - fr
        row = orc_vm.render(2048, 2048, 4096, 0, seed=SEED, y0=y, y1=y + 1, threads=16, **kw)[fr]
        assert bitwise_equal(img[fr], row).all(), fr


@pytest.mark.gpu
def test_config4_rank0_shard_full_size(gpu_tracer, orc_vm):
    """BASELINE configs[4]'s per-GPU workload at full size: rank 0's shard of the
    8-GPU render -- 16-row bands, band stride 8: 512 file rows of 4096 x 4096 x 8192 spp MIS, 1.7e10
    samples -- through the natural launch split (the 2^26-samples-per-workgroup bound, no lowered bound:
    2 launches), the auto layout at 8192 spp (64-sample chunks + taper, 137 chunks, 6.9 GB of partials)
    and the u32 queue guards.  The whole shard is finite and lit; two file rows (4096 x 8192 samples
    each) are recomputed by the oracle's pixel loop bit for bit (src/rt.cpp:786-800: every sample once,
    in order)."""
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    W = H = 4096
    spp, band, world = 8192, 16, 8
    img = gpu_tracer.render(width=W, height=H, spp=spp, estimator="mis", seed=SEED, fp64=True, band_rows=band,
                            band_stride=world, band_offset=0)
    assert img.shape == (H // world, W, 3)
    assert np.isfinite(img).all() and img.max() > 0
    for lr in (37, 470):  # shard rows -> file rows of rank 0's bands
        fr = (lr // band) * band * world + lr % band
        y = H - 1 - fr
        row = orc_vm.render(W, H, spp, 1, seed=SEED, y0=y, y1=y + 1, threads=16)[fr]
        assert bitwise_equal(img[lr], row).all(), (lr, fr)


def _set_launch_bound(tracer, log2):
    f = vpt.lib().vpt_debug_set_launch_bound
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    _lib.check(f(tracer._ctx, log2))


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,spp,log2,est,kw", [
    # 7 launches of 1792 units, the last one 512, at the 14 workgroups launch_pool clamps it to (tests/test_launch_plan.py)
    (32, 32, 96, 12, "ff", {}),
    (32, 32, 96, 12, "mis", dict(hg_g=0.5)),
    # configs[4]'s layout: 8192 spp -> 64-sample chunks + taper (137 chunks), split into 4 launches
    (8, 6, 8192, 14, "mis", {}),
])
def test_split_launches_equal_one_launch(gpu_tracer, orc_vm, w, h, spp, log2, est, kw):
    """The multi-launch path that BASELINE configs[4] takes on every GPU (2^34 samples per GPU > the
    2^26-samples-per-workgroup launch bound): the same render with the bound lowered
    (vpt_debug_set_launch_bound) so that it takes several launches, the last partial, equals the
    one-launch render and the oracle bit for bit (src/rt.cpp:786-800: every sample once, in order)."""
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    cfg = dict(width=w, height=h, spp=spp, estimator=est, seed=SEED + 5, fp64=True, **kw)
    one = gpu_tracer.render(**cfg)
    _set_launch_bound(gpu_tracer, log2)
    try:
        split = gpu_tracer.render(**cfg)
    finally:
        _set_launch_bound(gpu_tracer, 26)
    assert bitwise_equal(split, one).all()
    ref = orc_vm.render(w, h, spp, {"ff": 0, "mis": 1}[est], seed=SEED + 5, threads=16, **kw)
    assert bitwise_equal(split, ref).all()
    with pytest.raises(vpt.VPTError):
        _set_launch_bound(gpu_tracer, 27)


# ---------------------------------------------------------------- estimators 2-4
# explicitVPTracerRecursiveFree (2), implicitVPTracerRecursiveFree (3), explicitVPTracerRecursive
# (4): include/vptShadeMethods.h:1153, :940, :1014.
from scenes import EST_SCENES  # noqa: E402

EST234 = {2: "explicit_free", 3: "implicit_free", 4: "explicit"}


@pytest.mark.gpu
@pytest.mark.parametrize("scene", list(EST_SCENES))
@pytest.mark.parametrize("est", [2, 3, 4])
def test_trace_batch_vs_oracle_bitwise_e234(gpu_tracer, orc_vm, samples_e234, scene, est):
    sc = samples_e234[f"{scene}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    k = f"{scene}__e{est}__"
    rays, st = samples_e234[k + "ray"], samples_e234[k + "state1"]
    L, s = gpu_tracer.trace(EST234[est], _rays(rays), st)
    Lo, so = orc_vm.trace(est, rays, st)
    assert np.array_equal(s, so)
    same = bitwise_equal(L, Lo)
    assert same.all(), f"{(~same.all(1)).sum()} of {len(L)} samples differ"


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["default", "big_light", "dielectric"])
@pytest.mark.parametrize("est", [2, 3, 4])
def test_trace_batch_vs_reference_e234(gpu_tracer, samples_e234, scene, est):
    """against the reference's own per-sample values (same statistics bar as estimators 0/1)"""
    sc = samples_e234[f"{scene}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    k = f"{scene}__e{est}__"
    L, s = gpu_tracer.trace(est, _rays(samples_e234[k + "ray"]), samples_e234[k + "state1"])
    ref = samples_e234[k + "L"]
    assert np.array_equal(s, samples_e234[k + "state2"])
    fin = np.isfinite(ref)
    assert np.array_equal(np.isnan(ref), np.isnan(L)) and np.array_equal(fin, np.isfinite(L))
    close = np.abs(L[fin] - ref[fin]) <= 1e-12 * np.maximum(np.abs(ref[fin]), 1e-300)
    assert close.all(), f"{(~close).sum()} values differ"


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["default", "big_light"])
@pytest.mark.parametrize("est", [2, 3, 4])
def test_render_vs_oracle_bitwise_e234(gpu_tracer, orc_vm, scene, est):
    sc = EST_SCENES[scene]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    g = gpu_tracer.render(width=40, height=28, spp=20, estimator=EST234[est], seed=SEED, fp64=True)
    o = orc_vm.render(40, 28, 20, est, seed=SEED)
    assert bitwise_equal(g, o).all()


@pytest.mark.gpu
@pytest.mark.parametrize("g,depth", [(0.5, 0), (0.0, 3)])
@pytest.mark.parametrize("est", [2, 3, 4])
def test_extensions_vs_oracle_e234(gpu_tracer, orc_vm, g, depth, est):
    sc = EST_SCENES["big_light"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    gp = gpu_tracer.render(width=24, height=16, spp=4, estimator=est, hg_g=g, max_depth=depth, sigma_a=0.01,
                           sigma_s=0.09, seed=3, fp64=True)
    o = orc_vm.render(24, 16, 4, est, hg_g=g, max_depth=depth, sigma_a=0.01, sigma_s=0.09, seed=3)
    assert bitwise_equal(gp, o).all()


@pytest.mark.gpu
def test_count_work_matches_oracle_e234(gpu_tracer, orc_vm):
    sc = EST_SCENES["big_light"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    for est in (2, 3, 4):
        t, it = gpu_tracer.count_work(vpt.RenderConfig(width=32, height=24, spp=4, estimator=est, seed=9))
        _, c = orc_vm.render(32, 24, 4, est, seed=9, counters=True)
        assert (t, it) == (c.tests, c.iterations)


# ---------------------------------------------------------------- alternate scenes x 5 estimators
from scenes import ALT_SCENES  # noqa: E402


@pytest.mark.gpu
@pytest.mark.parametrize("scene", list(ALT_SCENES))
@pytest.mark.parametrize("est", [0, 1, 2, 3, 4])
def test_alt_scenes_vs_oracle_bitwise(gpu_tracer, orc_vm, samples_alt, scene, est):
    sc = samples_alt[f"{scene}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    k = f"{scene}__e{est}__"
    rays, st = samples_alt[k + "ray"], samples_alt[k + "state1"]
    L, s = gpu_tracer.trace(est, _rays(rays), st)
    Lo, so = orc_vm.trace(est, rays, st)
    assert np.array_equal(s, so)
    assert bitwise_equal(L, Lo).all()
    g = gpu_tracer.render(width=24, height=20, spp=6, estimator=est, seed=SEED, fp64=True)
    assert bitwise_equal(g, orc_vm.render(24, 20, 6, est, seed=SEED)).all()


# ---------------------------------------------------------------- pool kernel work hand-out
@pytest.mark.gpu
@pytest.mark.parametrize("w,h,spp,chunk", [
    (37, 23, 40, 1),    # tile padding (37 x 23 is not a multiple of 8): invalid units are dropped
    (3, 200, 9, 2),     # narrow image, ragged last chunk (9 = 4 x 2 + 1)
    (1, 1, 100, 1),     # one pixel, 100 units: one workgroup, the unit ring refilled many times
    (64, 64, 1, 0),     # 4096 one-sample units over a grid clamped to ceil(4096 / POOL) workgroups
    (129, 65, 3, 3),    # one chunk per pixel, odd sizes
])
def test_pool_work_handout_vs_oracle(gpu_tracer, orc_vm, w, h, spp, chunk):
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    g = gpu_tracer.render(width=w, height=h, spp=spp, chunk_spp=chunk, seed=21, fp64=True)
    eff = chunk if chunk > 0 else None  # None: the auto (tapered) layout
    o = orc_vm.render(w, h, spp, 0, seed=21, chunk=eff, threads=4)
    assert g.shape == o.shape and bitwise_equal(g, o).all()


# ---------------------------------------------------------------- estimator 5: iterativePathTracer
E5_SCENES = list(EST_SCENES) + list(ALT_SCENES)


def _e5_scene(name):
    return (EST_SCENES.get(name) or ALT_SCENES[name])()


@pytest.mark.gpu
@pytest.mark.parametrize("scene", E5_SCENES)
def test_trace_batch_vs_oracle_bitwise_e5(gpu_tracer, orc_vm, samples_e5, scene):
    """include/shadeMethods.h:104 per sample: same draws, same bits as the oracle"""
    sc = samples_e5[f"{scene}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    k = f"{scene}__e5__"
    rays, st = samples_e5[k + "ray"], samples_e5[k + "state1"]
    L, s = gpu_tracer.iterativePathTracer(_rays(rays), st)
    Lo, so = orc_vm.trace(5, rays, st)
    assert np.array_equal(s, so)
    same = bitwise_equal(L, Lo)
    assert same.all(), f"{(~same.all(1)).sum()} of {len(L)} samples differ"


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["default", "dielectric", "alt_metal_walls"])
def test_trace_batch_vs_reference_e5(gpu_tracer, samples_e5, scene):
    """against the reference's own per-sample values: same draws, same bits (the device libm is
    glibc's)"""
    sc = samples_e5[f"{scene}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    k = f"{scene}__e5__"
    L, s = gpu_tracer.trace(5, _rays(samples_e5[k + "ray"]), samples_e5[k + "state1"])
    ref = samples_e5[k + "L"]
    assert np.array_equal(s, samples_e5[k + "state2"])
    same = bitwise_equal(L, ref)
    assert same.all(), f"{(~same.all(1)).sum()} of {len(L)} samples differ"


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["default", "big_light", "dielectric", "alt_open_space"])
def test_render_vs_oracle_bitwise_e5(gpu_tracer, orc_vm, scene):
    """estimator 5 on the pool kernel: chunk sums like the other estimators (auto: spp <= 32 is one
    chunk, the reference's order; explicit chunk_spp: uniform chunks), bit-exact vs the oracle's layout"""
    sc = _e5_scene(scene)
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    o = orc_vm.render(40, 28, 20, 5, seed=SEED, chunk=20)
    for chunk in (0, 7):
        g = gpu_tracer.render(width=40, height=28, spp=20, estimator="surface_pt", seed=SEED, fp64=True,
                              chunk_spp=chunk)
        assert bitwise_equal(g, o if chunk == 0 else orc_vm.render(40, 28, 20, 5, seed=SEED, chunk=7)).all()
    assert np.abs(o).sum() > 0


@pytest.mark.gpu
def test_render_vs_oracle_bitwise_e5_tapered(gpu_tracer, orc_vm):
    """70 spp: auto chunks of 32 with the tapered tail (csrc/vpt_chunks.h), as the oracle lays them out"""
    sc = _e5_scene("default")
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    g = gpu_tracer.render(width=24, height=16, spp=70, estimator="surface_pt", seed=SEED, fp64=True)
    assert bitwise_equal(g, orc_vm.render(24, 16, 70, 5, seed=SEED, chunk=None, threads=4)).all()


@pytest.mark.gpu
def test_render_shards_e5(gpu_tracer):
    """row bands compose to the whole image, bit for bit"""
    gpu_tracer.set_scene(vpt.default_scene())
    full = gpu_tracer.render(width=32, height=32, spp=3, estimator="surface_pt", seed=5, fp64=True)
    parts = [gpu_tracer.render(width=32, height=32, spp=3, estimator="surface_pt", seed=5, fp64=True, band_rows=8,
                               band_stride=2, band_offset=r) for r in range(2)]
    rows = [[fr for b in range(r, 4, 2) for fr in range(b * 8, b * 8 + 8)] for r in range(2)]
    for r in range(2):
        assert bitwise_equal(parts[r], full[rows[r]]).all()


@pytest.mark.gpu
def test_count_work_matches_oracle_e5(gpu_tracer, orc_vm):
    sc = EST_SCENES["big_light"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    t, it = gpu_tracer.count_work(vpt.RenderConfig(width=32, height=24, spp=4, estimator="surface_pt", seed=9))
    _, c = orc_vm.render(32, 24, 4, 5, seed=9, counters=True, chunk=4)
    assert (t, it) == (c.tests, c.iterations)


# ---------------------------------------------------------------- estimator 6: rayMarching3
E6_CASES = ["default_l8", "default_l7", "alt_metal_walls_l7", "alt_open_space_l4", "alt_light_near_camera_l2"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", E6_CASES)
def test_trace_batch_vs_oracle_bitwise_e6(gpu_tracer, orc_vm, samples_e6, case):
    """include/rayMarchingMethods.h:330 per sample: same bits as the oracle, no draw consumed"""
    sc = samples_e6[f"{case}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    step, light = samples_e6[f"{case}__march"]
    k = f"{case}__e6__"
    rays, st = samples_e6[k + "ray"], samples_e6[k + "state1"]
    L, s = gpu_tracer.rayMarching3(_rays(rays), st, 0.001, 0.0125, step, int(light))
    Lo, so = orc_vm.trace(6, rays, st, 0.001, 0.0125, march_step=step, march_light=int(light))
    assert np.array_equal(s, so) and np.array_equal(s, st)
    same = bitwise_equal(L, Lo)
    assert same.all(), f"{(~same.all(1)).sum()} of {len(L)} samples differ"
    # against the reference's own values: the portable libm (exp, sqrt-based normalise) may differ
    # from glibc by an ulp, which moves no branch here but can move a last bit
    ref = samples_e6[k + "L"]
    assert (np.abs(L - ref) <= 1e-12 * np.maximum(np.abs(ref), 1e-300)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["default_l8", "alt_light_near_camera_l2"])
def test_render_vs_oracle_bitwise_e6(gpu_tracer, orc_vm, samples_e6, case):
    sc = samples_e6[f"{case}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    step, light = samples_e6[f"{case}__march"]
    g = gpu_tracer.render(width=24, height=24, spp=2, estimator="ray_marching", sigma_a=0.001, sigma_s=0.0125,
                          march_step=float(step), march_light=int(light), seed=SEED, fp64=True)
    o = orc_vm.render(24, 24, 2, 6, 0.001, 0.0125, seed=SEED, chunk=2, march_step=step, march_light=int(light))
    assert bitwise_equal(g, o).all()
    ref = samples_e6[f"{case}__e6__fb24x24x2"]
    assert (np.abs(g - ref) <= 1e-12 * np.maximum(np.abs(ref), 1e-300)).all()


@pytest.mark.gpu
def test_count_work_matches_oracle_e6(gpu_tracer, orc_vm):
    sc = vpt.default_scene()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    cfg = vpt.RenderConfig(width=16, height=12, spp=2, estimator="ray_marching", march_step=0.5, march_light=8, seed=9)
    t, it = gpu_tracer.count_work(cfg)
    _, c = orc_vm.render(16, 12, 2, 6, seed=9, counters=True, chunk=2, march_step=0.5, march_light=8)
    assert (t, it) == (c.tests, c.iterations)


@pytest.mark.gpu
def test_ray_marching_invalid_arguments(gpu_tracer):
    gpu_tracer.set_scene(vpt.default_scene())
    for kw in (dict(march_step=0.0), dict(march_step=-1.0), dict(march_step=float("nan")), dict(march_light=10),
               dict(march_light=-1)):
        with pytest.raises(vpt.VPTError):
            gpu_tracer.render(width=8, height=8, spp=1, estimator="ray_marching", **kw)


@pytest.mark.gpu
def test_large_spp_auto_chunk(gpu_tracer, orc_vm):
    """above 4096 spp the auto chunk grows (vpt_auto_chunk: 5000 spp -> 40-sample chunks + taper);
    same sums as the oracle's layout"""
    sc = SCENES["default"]()
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    g = gpu_tracer.render(width=8, height=6, spp=5000, seed=12, fp64=True)
    o = orc_vm.render(8, 6, 5000, 0, seed=12, threads=4)
    assert bitwise_equal(g, o).all()


# ---- BASELINE.json configs at their exact sample counts and media (small images) ----
@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h,spp,kw", [
    # configs[2]: MIS (free flight + equi-angular), HG g = 0.5, the default medium, 1024 spp
    ("mis_hg_1024", 8, 6, 1024, dict(estimator=1, hg_g=0.5)),
    # configs[4]: MIS at 8192 spp -- the > 4096-spp chunk layout (128 chunks + taper, vpt_chunks.h)
    ("mis_8192", 4, 3, 8192, dict(estimator=1)),
    # configs[3]: dense medium (sigma_t 0.03, BASELINE/DESIGN), depth cap 8, 4096 spp
    ("dense_4096", 4, 3, 4096, dict(estimator=0, sigma_a=0.003, sigma_s=0.027, max_depth=8)),
])
def test_baseline_configs_vs_oracle(gpu_tracer, orc_vm, name, w, h, spp, kw):
    gpu_tracer.set_scene(vpt.default_scene())
    orc_vm.set_scene(vpt.default_scene())
    ref = orc_vm.render(w, h, spp, seed=SEED + 17, threads=8, **kw)
    g = gpu_tracer.render(width=w, height=h, spp=spp, seed=SEED + 17, fp64=True, **kw)
    assert bitwise_equal(g, ref).all(), (name, np.abs(g - ref).max())
    assert np.isfinite(g).all() and g.max() > 0, name  # light reaches the camera (dense: sigma_t 0.03)


# ---------------------------------------------------------------- estimators 7-9: rayMarching2,
# rayMarchingGlobal, rayMarching (include/rayMarchingMethods.h:262, :106, :34) and punctualVolumetric (:12)
def _e789_keys():
    path = os.path.join(GOLDEN, "samples_e789.npz")
    return sorted(k[:-len("__march")] for k in np.load(path).files if k.endswith("__march"))


E789_NAMES = {7: "ray_marching_sa", 8: "ray_marching_global", 9: "ray_marching_explicit"}


@pytest.mark.gpu
@pytest.mark.parametrize("case", _e789_keys())
def test_trace_batch_vs_reference_bitwise_e789(gpu_tracer, orc_vm, samples_e789, case):
    """per sample: the reference's own values and end states, bit for bit (glibc-exact device libm)"""
    sc = samples_e789[f"{case}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    orc_vm.set_scene(sc)
    est, step, light = samples_e789[f"{case}__march"]
    est, light = int(est), int(light)
    k = f"{case}__"
    rays, st = samples_e789[k + "ray"], samples_e789[k + "state1"]
    if est == 7:
        L, s = gpu_tracer.rayMarching2(_rays(rays), st, 0.001, 0.0125, step, light)
    elif est == 8:
        L, s = gpu_tracer.rayMarchingGlobal(_rays(rays), st, 0.001, 0.0125, step)
    else:
        L, s = gpu_tracer.trace(E789_NAMES[9], _rays(rays), st, 0.001, 0.0125, march_step=step)
    assert np.array_equal(s, samples_e789[k + "state2"])
    same = bitwise_equal(L, samples_e789[k + "L"])
    assert same.all(), f"{(~same.all(1)).sum()} of {len(L)} samples differ from the reference"
    Lo, so = orc_vm.trace(est, rays, st, 0.001, 0.0125, march_step=step, march_light=light)
    assert bitwise_equal(L, Lo).all() and np.array_equal(s, so)


@pytest.mark.gpu
@pytest.mark.parametrize("case", _e789_keys())
def test_render_vs_reference_bitwise_e789(gpu_tracer, samples_e789, case):
    sc = samples_e789[f"{case}__scene"].view(vpt.SPHERE_DTYPE)
    gpu_tracer.set_scene(sc)
    est, step, light = samples_e789[f"{case}__march"]
    g = gpu_tracer.render(width=16, height=16, spp=2, estimator=E789_NAMES[int(est)], sigma_a=0.001, sigma_s=0.0125,
                          march_step=float(step), march_light=int(light), seed=SEED, fp64=True)
    assert bitwise_equal(g, samples_e789[f"{case}__fb16x16x2"]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("est", [7, 8, 9])
def test_count_work_matches_oracle_e789(gpu_tracer, orc_vm, est):
    from scenes import ALT_SCENES
    sc = ALT_SCENES["alt_area_light"]()
    gpu_tracer.set_scene(sc.view(vpt.SPHERE_DTYPE))
    orc_vm.set_scene(sc)
    step = 0.75 if est == 7 else 5.0
    cfg = vpt.RenderConfig(width=16, height=12, spp=2, estimator=E789_NAMES[est], march_step=step, march_light=5,
                           sigma_a=0.001, sigma_s=0.0125, seed=9)
    t, it = gpu_tracer.count_work(cfg)
    _, c = orc_vm.render(16, 12, 2, est, 0.001, 0.0125, seed=9, counters=True, chunk=2, march_step=step, march_light=5)
    assert (t, it) == (c.tests, c.iterations) and it > 0


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["default", "mat3", "point_lights"])
def test_punctual_volumetric_vs_reference_bitwise(gpu_tracer, samples_e789, scene):
    gpu_tracer.set_scene(samples_e789[f"pv_{scene}__scene"].view(vpt.SPHERE_DTYPE))
    ids, xs, want = samples_e789[f"pv_{scene}__id"], samples_e789[f"pv_{scene}__x"], samples_e789[f"pv_{scene}__out"]
    got = np.concatenate([gpu_tracer.punctualVolumetric(int(i), xs[ids == i], 1 / (4 * np.pi), 0.0135, 0.0125)
                          for i in np.unique(ids)])
    order = np.concatenate([np.nonzero(ids == i)[0] for i in np.unique(ids)])
    assert bitwise_equal(got, want[order]).all()


@pytest.mark.gpu
def test_ray_marching_out_parameters_vs_reference(gpu_tracer, samples_e789):
    from scenes import ALT_SCENES
    gpu_tracer.set_scene(ALT_SCENES["alt_area_light"]().view(vpt.SPHERE_DTYPE))
    rays, s1 = samples_e789["rmx__ray"], samples_e789["rmx__state1"]
    L, xn, ids, s2 = gpu_tracer.rayMarching(_rays(rays), s1, 0.0135, 0.0125, 7.0, x_new=samples_e789["rmx__xin"],
                                            idsource=-1)
    want = samples_e789["rmx__out"]
    assert bitwise_equal(L, want[:, :3]).all() and bitwise_equal(xn, want[:, 3:]).all()
    assert np.array_equal(ids, samples_e789["rmx__id"]) and np.array_equal(s2, samples_e789["rmx__state2"])
    assert (ids == -1).any() and (ids >= 0).any()


@pytest.mark.gpu
def test_ray_marching_789_invalid_arguments(gpu_tracer):
    gpu_tracer.set_scene(vpt.default_scene())
    for est in ("ray_marching_sa", "ray_marching_global", "ray_marching_explicit"):
        for kw in (dict(march_step=0.0), dict(march_step=float("inf"))):
            with pytest.raises(vpt.VPTError):
                gpu_tracer.render(width=8, height=8, spp=1, estimator=est, **kw)
    with pytest.raises(vpt.VPTError):
        gpu_tracer.render(width=8, height=8, spp=1, estimator="ray_marching_sa", march_light=10)
    gpu_tracer.set_scene(vpt.default_scene()[[0, 1, 2, 3, 7]])  # sphere 5 (hard-coded by rayMarching) missing
    for est in ("ray_marching_global", "ray_marching_explicit"):
        with pytest.raises(vpt.VPTError):
            gpu_tracer.render(width=8, height=8, spp=1, estimator=est, march_step=4.0)
    with pytest.raises(vpt.VPTError):
        gpu_tracer.punctualVolumetric(7, np.zeros((1, 3)), 0.1, 0.01, 0.01)
    gpu_tracer.set_scene(vpt.default_scene())
