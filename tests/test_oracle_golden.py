"""The oracle (oracle/vpt_oracle.c, libm build) against the reference's own outputs
(tests/golden/, generated from oracle/_ref/libvpt_ref.so by tests/golden/make_golden.py).

Bar: bit-exact for the free-flight estimator, every primitive and every random-state
trajectory; the MIS estimator within 1e-12 relative (the reference evaluates its linear recursion
back to front, the oracle front to back -- same terms, reassociated sums)."""
import numpy as np
import pytest
from conftest import bitwise_equal
from scenes import SCENES, stream_state

SEED = 0x5EED0001


def _scene_bytes(samples, name):
    return samples[f"{name}__scene"]


@pytest.mark.parametrize("scene", list(SCENES))
@pytest.mark.parametrize("est", [0, 1])
def test_per_sample_vs_reference(samples, orc, scene, est):
    orc.set_scene(_scene_bytes(samples, scene))
    k = f"{scene}__e{est}__"
    # camera rays (src/rt.cpp:787): bit-exact, same draws
    rays = samples[k + "ray"]
    for i in range(0, len(rays), 7):
        r, s = orc.camera_ray(64, 64, int(samples[k + "x"][i]), int(samples[k + "y"][i]), int(samples[k + "state0"][i]))
        assert np.array_equal(r, rays[i]) and s == int(samples[k + "state1"][i])
    L, st = orc.trace(est, rays, samples[k + "state1"])
    ref = samples[k + "L"]
    assert np.array_equal(st, samples[k + "state2"]), "random draws consumed differ"
    if est == 0:
        eq = bitwise_equal(L, ref)
        assert eq.all(), f"{(~eq.all(1)).sum()} of {len(L)} samples differ"
    else:
        fin = np.isfinite(ref)
        assert np.array_equal(fin, np.isfinite(L))
        assert np.array_equal(np.isnan(ref), np.isnan(L))
        rel = np.abs(L[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
        assert rel.max(initial=0) <= 1e-12


@pytest.mark.parametrize("scene", list(SCENES))
@pytest.mark.parametrize("est", [0, 1])
def test_framebuffer_vs_reference(samples, orc, scene, est):
    orc.set_scene(_scene_bytes(samples, scene))
    ref = samples[f"{scene}__e{est}__fb24x24x4"]
    out = orc.render(24, 24, 4, est, seed=SEED, threads=2)
    if est == 0:
        assert bitwise_equal(out, ref).all()
    else:
        fin = np.isfinite(ref)
        assert np.array_equal(fin, np.isfinite(out))
        np.testing.assert_allclose(out[fin], ref[fin], rtol=1e-12, atol=1e-300)


def test_stream_state_spec(orc, samples):
    # three independent statements of the per-sample stream key agree
    for idx, i in [(0, 0), (1, 0), (0, 1), (4095, 15), (16777215, 8191), (123456, 77)]:
        assert orc.stream_state(SEED, idx, i) == stream_state(SEED, idx, i)
    k = "default__e0__"
    for j in range(0, 64):
        x, y, s = int(samples[k + "x"][j]), int(samples[k + "y"][j]), int(samples[k + "sample"][j])
        assert int(samples[k + "state0"][j]) == stream_state(SEED, (63 - y) * 64 + x, s)


def test_default_scene_bytes(samples):
    import os
    from conftest import GOLDEN

    ref = np.load(os.path.join(GOLDEN, "default_scene.npy"))
    assert np.array_equal(ref, SCENES["default"]().view(np.uint8))
    assert np.array_equal(ref, samples["default__scene"])


# ---------------------------------------------------------------- primitives
def _v(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def test_primitives_geometry(orc, prims):
    orc.set_scene(SCENES["default"]())
    f = orc.prim
    rays = _v(prims["ray"])
    n = len(rays)
    si = np.array([[f("sphere_intersect")(i, rays[k].ctypes.data) for i in range(10)] for k in range(n)])
    assert bitwise_equal(si, prims["sphere_intersect"]).all()
    for k in range(n):
        t = np.zeros(1)
        idv = np.zeros(1, dtype=np.int32)
        hit = f("intersect")(rays[k].ctypes.data, t.ctypes.data, idv.ctypes.data)
        assert hit == prims["intersect_hit"][k] and t[0] == prims["intersect_t"][k] and idv[0] == prims["intersect_id"][k]
    L, X = _v(prims["vis_light"]), _v(prims["vis_x"])
    vis = [f("visibility")(L[k].ctypes.data, X[k].ctypes.data) for k in range(n)]
    assert np.array_equal(vis, prims["visibility"])
    tr = [f("transmitance")(X[k].ctypes.data, L[k].ctypes.data, 0.01) for k in range(n)]
    assert np.array_equal(tr, prims["transmitance"])
    nn = _v(prims["n"])
    cs = np.zeros((n, 6))
    for k in range(n):
        f("coordinate_system")(nn[k].ctypes.data, cs[k, :3].ctypes.data, cs[k, 3:].ctypes.data)
    assert np.array_equal(cs, prims["coordinate_system"])


def test_primitives_sampling(orc, prims):
    f = orc.prim
    nn, st, cm = _v(prims["n"]), prims["state"], prims["cmax"]
    n = len(nn)
    calls = {
        "solid_angle_dir": lambda k, o: f("solid_angle_dir")(nn[k].ctypes.data, cm[k], int(st[k]), o.ctypes.data),
        "cosine_hemispheric": lambda k, o: f("cosine_hemispheric")(nn[k].ctypes.data, int(st[k]), o.ctypes.data),
        "isotropic_phase": lambda k, o: f("isotropic_phase")(int(st[k]), o.ctypes.data),
        "vector_facet": lambda k, o: f("vector_facet")(0.09, int(st[k]), o.ctypes.data),
    }
    for name, call in calls.items():
        v = np.zeros((n, 3))
        s = np.array([call(k, v[k]) for k in range(n)], dtype=np.uint64)
        assert np.array_equal(s, prims[name + "_state"]), name
        assert bitwise_equal(v, prims[name]).all(), name


def test_primitives_microfacet(orc, prims):
    f = orc.prim
    n = len(prims["cw"])
    eta, kappa = _v([1.66058, 0.88143, 0.521467]), _v([9.2282, 6.27077, 4.83803])
    fr = np.zeros((n, 3))
    for k in range(n):
        f("fresnel")(prims["cw"][k], eta.ctypes.data, kappa.ctypes.data, fr[k].ctypes.data)
    assert bitwise_equal(fr, prims["fresnel"]).all()
    wi, wo, wh = _v(prims["wi"]), _v(prims["wo"]), _v(prims["wh"])
    zn = _v(np.tile([0, 0, 1.0], (n, 1)))
    fm = np.zeros((n, 3))
    for k in range(n):
        f("fr_microfacet")(eta.ctypes.data, kappa.ctypes.data, wi[k].ctypes.data, wh[k].ctypes.data, wo[k].ctypes.data,
                           0.09, zn[k].ctypes.data, fm[k].ctypes.data)
    assert bitwise_equal(fm, prims["fr_microfacet"]).all()
    mp = [f("microfacet_prob")(wo[k].ctypes.data, wh[k].ctypes.data, 0.09, zn[k].ctypes.data) for k in range(n)]
    assert bitwise_equal(mp, prims["microfacet_prob"]).all()


def test_primitives_shading(orc, prims):
    orc.set_scene(SCENES["default"]())
    f = orc.prim
    objs, xs, ns, wr, st = prims["obj"], _v(prims["xs"]), _v(prims["ns"]), _v(prims["wray"]), prims["state"]
    n = len(objs)
    I8, L8 = _v([6000, 0, 0.0]), _v([-23, 24.3, 0.0])
    pl = np.zeros((n, 3))
    ms, mss = np.zeros((n, 3)), np.zeros(n, dtype=np.uint64)
    bf, bw, bp, bs = np.zeros((n, 3)), np.zeros((n, 3)), np.zeros(n), np.zeros(n, dtype=np.uint64)
    for k in range(n):
        f("plight")(int(objs[k]), xs[k].ctypes.data, ns[k].ctypes.data, wr[k].ctypes.data, I8.ctypes.data,
                    L8.ctypes.data, 0.09, pl[k].ctypes.data)
        mss[k] = f("misv2")(int(objs[k]), xs[k].ctypes.data, ns[k].ctypes.data, wr[k].ctypes.data, 0.09, 0.01,
                            int(st[k]), ms[k].ctypes.data)
        pr = np.zeros(1)
        bs[k] = f("bdsf")(wr[k].ctypes.data, ns[k].ctypes.data, int(objs[k]), int(st[k]), bf[k].ctypes.data,
                          bw[k].ctypes.data, pr.ctypes.data)
        bp[k] = pr[0]
    assert bitwise_equal(pl, prims["plight"]).all()
    assert np.array_equal(mss, prims["misv2_state"]) and bitwise_equal(ms, prims["misv2"]).all()
    assert np.array_equal(bs, prims["bdsf_state"])
    assert bitwise_equal(bf, prims["bdsf_fs"]).all() and bitwise_equal(bw, prims["bdsf_wi"]).all()
    assert bitwise_equal(bp, prims["bdsf_prob"]).all()


def test_primitives_media(orc, prims):
    orc.set_scene(SCENES["default"]())
    f = orc.prim
    X, src, st, rays = _v(prims["vis_x"]), prims["src"], prims["state"], _v(prims["ray"])
    n = len(src)
    fss, ssv = np.zeros((n, 3)), np.zeros((n, 3))
    eq = np.zeros((n, 5))
    for k in range(n):
        s1 = f("free_single_scattering")(X[k].ctypes.data, int(src[k]), 0.01, 1 / 3, int(st[k]), fss[k].ctypes.data)
        s2 = f("single_scattering")(X[k].ctypes.data, int(src[k]), 0.01, 0.009, 0.7, 1 / 3, int(st[k]), ssv[k].ctypes.data)
        s3 = f("equiangular_params2")(int(src[k]), prims["tmax"][k], rays[k].ctypes.data, eq[k].ctypes.data, int(st[k]))
        assert s1 == prims["free_single_scattering_state"][k]
        assert s2 == prims["single_scattering_state"][k]
        assert s3 == prims["equiangular_params2_state"][k]
    assert bitwise_equal(fss, prims["free_single_scattering"]).all()
    assert bitwise_equal(ssv, prims["single_scattering"]).all()
    assert bitwise_equal(eq, prims["equiangular_params2"]).all()
    ep = [f("equiangular_prob")(*eq[k, 1:]) for k in range(n)]
    assert bitwise_equal(ep, prims["equiangular_prob"]).all()


def test_to_display(orc, prims):
    got = [orc.prim("to_display")(v) for v in prims["disp_in"]]
    assert np.array_equal(got, prims["to_display"])


# ---- the other estimators: explicitVPTracerRecursiveFree (2),
# implicitVPTracerRecursiveFree (3), explicitVPTracerRecursive (4), include/vptShadeMethods.h:1153,
# :940, :1014.  All recursive: same draws bit-for-bit, values within 1e-12 relative (H14).
from scenes import EST_SCENES  # noqa: E402


def _close_nan_aware(out, ref, rtol=1e-12):
    assert np.array_equal(np.isnan(ref), np.isnan(out))
    fin = np.isfinite(ref)
    assert np.array_equal(fin, np.isfinite(out))
    rel = np.abs(out[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
    assert rel.max(initial=0) <= rtol


@pytest.mark.parametrize("scene", list(EST_SCENES))
@pytest.mark.parametrize("est", [2, 3, 4])
def test_per_sample_vs_reference_e234(samples_e234, orc, scene, est):
    orc.set_scene(samples_e234[f"{scene}__scene"])
    k = f"{scene}__e{est}__"
    L, st = orc.trace(est, samples_e234[k + "ray"], samples_e234[k + "state1"])
    assert np.array_equal(st, samples_e234[k + "state2"]), "random draws consumed differ"
    _close_nan_aware(L, samples_e234[k + "L"])


@pytest.mark.parametrize("scene", list(EST_SCENES))
@pytest.mark.parametrize("est", [2, 3, 4])
def test_framebuffer_vs_reference_e234(samples_e234, orc, scene, est):
    orc.set_scene(samples_e234[f"{scene}__scene"])
    out = orc.render(24, 24, 4, est, seed=SEED, threads=2, chunk=4)  # chunk = spp: the reference's order
    _close_nan_aware(out, samples_e234[f"{scene}__e{est}__fb24x24x4"])


def test_explicit_free_is_the_free_flight_loop(samples_e234, orc):
    """the recursive FF twin equals iterativeVPTracerFree up to reassociation -- same
    draws, same branches, values within 1e-12."""
    orc.set_scene(samples_e234["default__scene"])
    k = "default__e2__"
    L0, s0 = orc.trace(0, samples_e234[k + "ray"], samples_e234[k + "state1"])
    assert np.array_equal(s0, samples_e234[k + "state2"])
    _close_nan_aware(L0, samples_e234[k + "L"])


# ---- the reference's alternate scenes (include/Sphere.cpp:27-105) through all five estimators
from scenes import ALT_SCENES  # noqa: E402


@pytest.mark.parametrize("scene", list(ALT_SCENES))
@pytest.mark.parametrize("est", [0, 1, 2, 3, 4])
def test_alt_scenes_vs_reference(samples_alt, orc, scene, est):
    orc.set_scene(samples_alt[f"{scene}__scene"])
    k = f"{scene}__e{est}__"
    L, st = orc.trace(est, samples_alt[k + "ray"], samples_alt[k + "state1"])
    assert np.array_equal(st, samples_alt[k + "state2"]), "random draws consumed differ"
    if est == 0:
        assert bitwise_equal(L, samples_alt[k + "L"]).all()
    else:
        _close_nan_aware(L, samples_alt[k + "L"])
    out = orc.render(24, 24, 4, est, seed=SEED, threads=2, chunk=4)
    if est == 0:
        assert bitwise_equal(out, samples_alt[k + "fb24x24x4"]).all()
    else:
        _close_nan_aware(out, samples_alt[k + "fb24x24x4"])


# ---- iterativePathTracer (include/shadeMethods.h:104): surface-only estimator 5
from scenes import EST_SCENES  # noqa: E402

E5_SCENES = list(EST_SCENES) + list(ALT_SCENES)


@pytest.mark.parametrize("scene", E5_SCENES)
def test_surface_pt_vs_reference(samples_e5, orc, scene):
    """same draws and the same bits as the reference (MIS = MISv2 without the transmitance factor,
    BDSF = bdsf, pLight over every r == 0 sphere), per sample and on a 24x24x4 framebuffer"""
    orc.set_scene(samples_e5[f"{scene}__scene"])
    k = f"{scene}__e5__"
    L, st = orc.trace(5, samples_e5[k + "ray"], samples_e5[k + "state1"])
    assert np.array_equal(st, samples_e5[k + "state2"]), "random draws consumed differ"
    assert bitwise_equal(L, samples_e5[k + "L"]).all()
    out = orc.render(24, 24, 4, 5, seed=SEED, threads=2, chunk=4)  # chunk = spp: the reference's order
    assert bitwise_equal(out, samples_e5[k + "fb24x24x4"]).all()
    # the fixture exercises the path -- except where the reference's own tests make the image black:
    # no emitter, or (alt_area_light) a light with radiance.x == 0, which iterativePathTracer and MIS
    # never treat as a light (include/shadeMethods.h:122, include/misSamplingFunctions.h:29)
    assert (samples_e5[k + "L"] != 0).any() == (scene not in ("no_emitter", "alt_area_light"))


# ---- rayMarching3 (include/rayMarchingMethods.h:330): estimator 6, no random draw past the camera jitter
E6_CASES = ["default_l8", "default_l7", "alt_metal_walls_l7", "alt_open_space_l4", "alt_light_near_camera_l2"]


@pytest.mark.parametrize("case", E6_CASES)
def test_ray_marching_vs_reference(samples_e6, orc, case):
    orc.set_scene(samples_e6[f"{case}__scene"])
    step, light = samples_e6[f"{case}__march"]
    k = f"{case}__e6__"
    L, st = orc.trace(6, samples_e6[k + "ray"], samples_e6[k + "state1"], 0.001, 0.0125, march_step=step,
                      march_light=int(light))
    assert np.array_equal(st, samples_e6[k + "state1"]) and np.array_equal(st, samples_e6[k + "state2"])
    assert bitwise_equal(L, samples_e6[k + "L"]).all()
    out = orc.render(24, 24, 2, 6, 0.001, 0.0125, seed=SEED, threads=2, chunk=2, march_step=step,
                     march_light=int(light))
    assert bitwise_equal(out, samples_e6[k + "fb24x24x2"]).all()
    # light 7 of the default scene is a sphere light (r = 2): its shadow rays start at its centre and
    # stop on its own surface, so the reference's marching sees it nowhere
    assert (np.abs(out).sum() > 0) == (case != "default_l7")


# ---- rayMarching2 (:262, estimator 7), rayMarchingGlobal (:106, estimator 8), rayMarching (:34,
# estimator 9) of include/rayMarchingMethods.h: same draws, bit-exact values, per sample and 16x16x2
def _e789_keys():
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "samples_e789.npz")
    return sorted(k[:-len("__march")] for k in np.load(path).files if k.endswith("__march"))


@pytest.mark.parametrize("case", _e789_keys())
def test_ray_marching_789_vs_reference(samples_e789, orc, case):
    orc.set_scene(samples_e789[f"{case}__scene"])
    est, step, light = samples_e789[f"{case}__march"]
    est, light = int(est), int(light)
    k = f"{case}__"
    L, st = orc.trace(est, samples_e789[k + "ray"], samples_e789[k + "state1"], 0.001, 0.0125, march_step=step,
                      march_light=light)
    assert np.array_equal(st, samples_e789[k + "state2"])
    assert bitwise_equal(L, samples_e789[k + "L"]).all()
    out = orc.render(16, 16, 2, est, 0.001, 0.0125, seed=SEED, threads=2, chunk=2, march_step=step,
                     march_light=light)
    assert bitwise_equal(out, samples_e789[k + "fb16x16x2"]).all()
    # every case draws (solid-angle samples); the default scene's sphere 5 is the unlit metal sphere,
    # so rayMarching sees no light there (rayMarchingGlobal still returns the lights the camera sees)
    assert not np.array_equal(samples_e789[k + "state1"], samples_e789[k + "state2"])
    assert (np.abs(out).sum() > 0) == (not (est == 9 and "default" in case))


@pytest.mark.parametrize("scene", ["default", "mat3", "point_lights"])
def test_punctual_volumetric_vs_reference(samples_e789, orc, scene):
    """punctualVolumetric (include/rayMarchingMethods.h:12-31): visibilityVPT + multipleT"""
    orc.set_scene(samples_e789[f"pv_{scene}__scene"])
    ids, xs, want = samples_e789[f"pv_{scene}__id"], samples_e789[f"pv_{scene}__x"], samples_e789[f"pv_{scene}__out"]
    got = np.zeros_like(want)
    f = orc.prim("punctual_volumetric")
    for k in range(len(ids)):
        f(int(ids[k]), np.ascontiguousarray(xs[k]).ctypes.data, 1 / (4 * np.pi), 0.0135, 0.0125, got[k].ctypes.data)
    assert bitwise_equal(got, want).all()
    assert (want != 0).any() and (want == 0).all(axis=1).any()  # lit and shadowed points both present


def test_ray_marching_out_parameters_vs_reference(samples_e789, orc):
    """rayMarching's x_new / idsource (include/rayMarchingMethods.h:41-44): set on a hit, kept on a miss"""
    import ctypes
    from scenes import ALT_SCENES
    orc.set_scene(ALT_SCENES["alt_area_light"]())
    rays, s1, xin = samples_e789["rmx__ray"], samples_e789["rmx__state1"], samples_e789["rmx__xin"]
    out = np.zeros((len(rays), 6))
    ids = np.zeros(len(rays), dtype=np.int32)
    s2 = np.zeros(len(rays), dtype=np.uint64)
    f = orc.prim("ray_marching_explicit")
    for k in range(len(rays)):
        idk = ctypes.c_int(-1)
        s2[k] = f(np.ascontiguousarray(rays[k]).ctypes.data, 0.0135, 0.0125, 7.0, int(s1[k]), xin.ctypes.data,
                  ctypes.byref(idk), out[k].ctypes.data)
        ids[k] = idk.value
    assert bitwise_equal(out, samples_e789["rmx__out"]).all()
    assert np.array_equal(ids, samples_e789["rmx__id"]) and np.array_equal(s2, samples_e789["rmx__state2"])
    assert (ids == -1).any() and (ids >= 0).any()
