#!/usr/bin/env python3
"""Generates the committed golden fixtures from the REFERENCE's own functions.

Runs oracle/_ref/libvpt_ref.so (ref_harness.cpp: the reference's headers compiled in place from
/root/reference, driven with per-sample erand48 states) and, for the file-format check, the
reference program oracle/_ref/rt itself.  Only inputs and outputs are stored (no reference
source).  The reference has no tests or golden vectors of its own, so these are the
pins of the oracle.

    python tests/golden/make_golden.py          # writes tests/golden/*.npz, *.json
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle.oracle import Reference  # noqa: E402
from scenes import ALT_SCENES, EST_SCENES, SCENES, stream_state  # noqa: E402

SEED = 0x5EED0001
W = H = 64


def per_sample(ref: Reference, est: int, n: int, rng) -> dict:
    xs = rng.integers(0, W, n)
    ys = rng.integers(0, H, n)
    si = rng.integers(0, 1 << 20, n)
    s0 = np.array([stream_state(SEED, int((H - y - 1) * W + x), int(i)) for x, y, i in zip(xs, ys, si)], dtype=np.uint64)
    rays = np.zeros((n, 6))
    s1 = np.zeros(n, dtype=np.uint64)
    for k in range(n):
        s1[k] = ref.prim("camera_ray")(W, H, int(xs[k]), int(ys[k]), int(s0[k]), rays[k].ctypes.data)
    out, s2 = ref.trace(est, rays, s1)
    return dict(x=xs, y=ys, sample=si, state0=s0, ray=rays, state1=s1, L=out, state2=s2)


def prim_kats(ref: Reference, rng, n=400) -> dict:
    P = lambda a: np.ascontiguousarray(a, dtype=np.float64)  # noqa: E731
    f = ref.prim
    d = {}
    unit = lambda k: (lambda v: v / np.linalg.norm(v, axis=-1, keepdims=True))(rng.normal(size=(k, 3)))  # noqa: E731
    # rays from inside the room, random directions
    o = rng.uniform([-45, -38, -78], [45, 38, 200], size=(n, 3))
    dd = unit(n)
    rays = P(np.concatenate([o, dd], 1))
    d["ray"] = rays
    d["sphere_intersect"] = np.array([[f("sphere_intersect")(i, rays[k].ctypes.data) for i in range(10)] for k in range(n)])
    t = np.zeros(n)
    ids = np.zeros(n, dtype=np.int32)
    hit = np.zeros(n, dtype=np.int32)
    for k in range(n):
        tt = np.zeros(1)
        ii = np.zeros(1, dtype=np.int32)
        hit[k] = f("intersect")(rays[k].ctypes.data, tt.ctypes.data, ii.ctypes.data)
        t[k], ids[k] = tt[0], ii[0]
    d["intersect_hit"], d["intersect_t"], d["intersect_id"] = hit, t, ids
    lights = P(np.array([[-23, 24.3, 0.0], [0, 24.3, -35.0], [23, 24.3, 35.0]])[rng.integers(0, 3, n)])
    d["vis_light"], d["vis_x"] = lights, P(o)
    d["visibility"] = np.array([f("visibility")(lights[k].ctypes.data, o[k].ctypes.data) for k in range(n)])
    d["transmitance"] = np.array([f("transmitance")(o[k].ctypes.data, lights[k].ctypes.data, 0.01) for k in range(n)])
    nn = P(unit(n))
    d["n"] = nn
    cs = np.zeros((n, 6))
    for k in range(n):
        f("coordinate_system")(nn[k].ctypes.data, cs[k, :3].ctypes.data, cs[k, 3:].ctypes.data)
    d["coordinate_system"] = cs
    states = np.array([int(x) for x in rng.integers(0, 1 << 48, n, dtype=np.int64)], dtype=np.uint64)
    d["state"] = states
    cm = rng.uniform(0.5, 1.0, n)
    cm[:20] = 1.0
    d["cmax"] = cm
    for name, call in [
        ("solid_angle_dir", lambda k, out: f("solid_angle_dir")(nn[k].ctypes.data, cm[k], int(states[k]), out.ctypes.data)),
        ("cosine_hemispheric", lambda k, out: f("cosine_hemispheric")(nn[k].ctypes.data, int(states[k]), out.ctypes.data)),
        ("isotropic_phase", lambda k, out: f("isotropic_phase")(int(states[k]), out.ctypes.data)),
        ("vector_facet", lambda k, out: f("vector_facet")(0.09, int(states[k]), out.ctypes.data)),
    ]:
        v = np.zeros((n, 3))
        s = np.zeros(n, dtype=np.uint64)
        for k in range(n):
            s[k] = call(k, v[k])
        d[name], d[name + "_state"] = v, s
    cw = rng.uniform(-1, 1, n)
    d["cw"] = cw
    eta, kappa = P([1.66058, 0.88143, 0.521467]), P([9.2282, 6.27077, 4.83803])
    fr = np.zeros((n, 3))
    for k in range(n):
        f("fresnel")(cw[k], eta.ctypes.data, kappa.ctypes.data, fr[k].ctypes.data)
    d["fresnel"] = fr
    wi, wo = P(unit(n)), P(unit(n))
    wh = P((lambda v: v / np.linalg.norm(v, axis=1, keepdims=True))(wi + wo))
    zn = P(np.tile([0, 0, 1.0], (n, 1)))
    d["wi"], d["wo"], d["wh"] = wi, wo, wh
    fm = np.zeros((n, 3))
    for k in range(n):
        f("fr_microfacet")(eta.ctypes.data, kappa.ctypes.data, wi[k].ctypes.data, wh[k].ctypes.data, wo[k].ctypes.data, 0.09,
                           zn[k].ctypes.data, fm[k].ctypes.data)
    d["fr_microfacet"] = fm
    d["microfacet_prob"] = np.array([f("microfacet_prob")(wo[k].ctypes.data, wh[k].ctypes.data, 0.09, zn[k].ctypes.data)
                                     for k in range(n)])
    # surface points on the scene's spheres with outward normals and incoming directions
    objs = rng.integers(0, 7, n)
    cen = P(np.array([[-1e5 - 49, 0, 0], [1e5 + 49, 0, 0], [0, 0, -1e5 - 81.6], [0, -1e5 - 40.8, 0], [0, 1e5 + 40.8, 0],
                      [-23, -24.3, -34.6], [23, -24.3, -3.6]])[objs])
    rad = np.array([1e5] * 5 + [16.5, 16.5])[objs]
    u = unit(n)
    xsurf = cen + rad[:, None] * u
    xsurf = np.where(objs[:, None] < 5, np.clip(xsurf, [-49, -40.8, -81.6], [49, 40.8, 200]), xsurf)
    nsurf = xsurf - cen
    nsurf = nsurf / np.sqrt((nsurf * nsurf).sum(1, keepdims=True))
    wray = unit(n)
    wray = np.where(((wray * nsurf).sum(1) > 0)[:, None], -wray, wray)
    xsurf, nsurf, wray = P(xsurf), P(nsurf), P(wray)
    d["obj"], d["xs"], d["ns"], d["wray"] = objs.astype(np.int32), xsurf, nsurf, wray
    pl = np.zeros((n, 3))
    I8, L8 = P([6000, 0, 0.0]), P([-23, 24.3, 0.0])
    for k in range(n):
        f("plight")(int(objs[k]), xsurf[k].ctypes.data, nsurf[k].ctypes.data, wray[k].ctypes.data, I8.ctypes.data,
                    L8.ctypes.data, 0.09, pl[k].ctypes.data)
    d["plight"] = pl
    ms, mss = np.zeros((n, 3)), np.zeros(n, dtype=np.uint64)
    bf, bw, bp, bs = np.zeros((n, 3)), np.zeros((n, 3)), np.zeros(n), np.zeros(n, dtype=np.uint64)
    for k in range(n):
        mss[k] = f("misv2")(int(objs[k]), xsurf[k].ctypes.data, nsurf[k].ctypes.data, wray[k].ctypes.data, 0.09, 0.01,
                            int(states[k]), ms[k].ctypes.data)
        pr = np.zeros(1)
        bs[k] = f("bdsf")(wray[k].ctypes.data, nsurf[k].ctypes.data, int(objs[k]), int(states[k]), bf[k].ctypes.data,
                          bw[k].ctypes.data, pr.ctypes.data)
        bp[k] = pr[0]
    d["misv2"], d["misv2_state"] = ms, mss
    d["bdsf_fs"], d["bdsf_wi"], d["bdsf_prob"], d["bdsf_state"] = bf, bw, bp, bs
    src = rng.choice([7, 8, 9], n).astype(np.int32)
    d["src"] = src
    fss, fsss = np.zeros((n, 3)), np.zeros(n, dtype=np.uint64)
    ssv, ssvs = np.zeros((n, 3)), np.zeros(n, dtype=np.uint64)
    for k in range(n):
        fsss[k] = f("free_single_scattering")(o[k].ctypes.data, int(src[k]), 0.01, 1 / 3, int(states[k]), fss[k].ctypes.data)
        ssvs[k] = f("single_scattering")(o[k].ctypes.data, int(src[k]), 0.01, 0.009, 0.7, 1 / 3, int(states[k]),
                                         ssv[k].ctypes.data)
    d["free_single_scattering"], d["free_single_scattering_state"] = fss, fsss
    d["single_scattering"], d["single_scattering_state"] = ssv, ssvs
    tmax = rng.uniform(1, 300, n)
    tmax[:10] = np.float64(np.float32(3.4028234663852886e38))
    d["tmax"] = tmax
    eq, eqs = np.zeros((n, 5)), np.zeros(n, dtype=np.uint64)
    for k in range(n):
        eqs[k] = f("equiangular_params2")(int(src[k]), tmax[k], rays[k].ctypes.data, eq[k].ctypes.data, int(states[k]))
    d["equiangular_params2"], d["equiangular_params2_state"] = eq, eqs
    d["equiangular_prob"] = np.array([f("equiangular_prob")(*eq[k, 1:]) for k in range(n)])
    vals = np.concatenate([np.linspace(-0.5, 1.5, 301), rng.uniform(0, 1, 200), [np.nan, np.inf, -np.inf]])
    d["disp_in"] = vals
    d["to_display"] = np.array([f("to_display")(v) for v in vals], dtype=np.int64)
    return d


def reference_program_ppm() -> dict:
    """Runs the reference program (`rt 1`, 1024x768, 1 spp) for the PPM format facts."""
    exe = os.path.join(ROOT, "oracle", "_ref", "rt")
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run([exe, "1"], cwd=td, capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, OMP_NUM_THREADS="8"))
        data = open(os.path.join(td, "image.ppm"), "rb").read()
    hdr_end = data.index(b"\n", data.index(b"\n", 3) + 1) + 1
    vals = np.array(data[hdr_end:].split(), dtype=np.int64)
    return {
        "stdout_prefix": r.stdout.split(":")[0],
        "header": data[:hdr_end].decode(),
        "bytes": len(data),
        "ends_with_space": data.endswith(b" "),
        "ends_with_newline": data.endswith(b"\n"),
        "n_values": int(len(vals)),
        "min": int(vals.min()),
        "max": int(vals.max()),
        "channel_mean_8bit": [float(vals[c::3].mean()) for c in range(3)],
        "spp": 1,
    }


def main():
    ref = Reference()
    rng = np.random.default_rng(20250523)
    # the reference's default scene bytes (include/Sphere.cpp:11-22)
    np.save(os.path.join(HERE, "default_scene.npy"), ref.default_scene())
    bundle = {}
    for name, mk in SCENES.items():
        sc = mk()
        ref.set_scene(sc)
        bundle[f"{name}__scene"] = sc.view(np.uint8)
        for est in (0, 1):
            n = 1024 if name == "default" else 384
            ps = per_sample(ref, est, n, rng)
            for k, v in ps.items():
                bundle[f"{name}__e{est}__{k}"] = v
            fb = ref.render(24, 24, 4, est, seed=SEED)
            bundle[f"{name}__e{est}__fb24x24x4"] = fb
    np.savez_compressed(os.path.join(HERE, "samples.npz"), **bundle)
    ref.set_scene(ref.default_scene())
    np.savez_compressed(os.path.join(HERE, "primitives.npz"), **prim_kats(ref, rng))
    # a slightly larger framebuffer for image-level statistics (default scene, both estimators)
    stats = {}
    for est in (0, 1):
        fb = ref.render(64, 64, 16, est, seed=SEED + 1)
        np.save(os.path.join(HERE, f"fb64x64x16_e{est}.npy"), fb.astype(np.float64))
        stats[f"e{est}_mean"] = fb.reshape(-1, 3).mean(0).tolist()
    with open(os.path.join(HERE, "reference_ppm.json"), "w") as f:
        json.dump({"program": reference_program_ppm(), "seed": SEED, "fb_stats": stats}, f, indent=1)
    print("wrote fixtures to", HERE)


def estimators_234():
    """Per-sample known answers and 24x24x4 framebuffers of the other three estimators
    (explicitVPTracerRecursiveFree, implicitVPTracerRecursiveFree, explicitVPTracerRecursive;
    include/vptShadeMethods.h:1153, :940, :1014) -> samples_e234.npz.  Own RNG seed, so the
    estimator 0/1 fixtures above stay byte-identical."""
    ref = Reference()
    rng = np.random.default_rng(20261015)
    bundle = {}
    for name, mk in EST_SCENES.items():
        sc = mk()
        ref.set_scene(sc)
        bundle[f"{name}__scene"] = sc.view(np.uint8)
        for est in (2, 3, 4):
            ps = per_sample(ref, est, 384, rng)
            for k, v in ps.items():
                bundle[f"{name}__e{est}__{k}"] = v
            bundle[f"{name}__e{est}__fb24x24x4"] = ref.render(24, 24, 4, est, seed=SEED)
    np.savez_compressed(os.path.join(HERE, "samples_e234.npz"), **bundle)
    print("wrote", os.path.join(HERE, "samples_e234.npz"))


def alt_scenes():
    """The reference's alternate scenes (commented out in include/Sphere.cpp:27-105, restated in
    tests/scenes.py ALT_SCENES) through all five estimators -> samples_alt.npz."""
    ref = Reference()
    rng = np.random.default_rng(20261016)
    bundle = {}
    for name, mk in ALT_SCENES.items():
        sc = mk()
        ref.set_scene(sc)
        bundle[f"{name}__scene"] = sc.view(np.uint8)
        for est in range(5):
            ps = per_sample(ref, est, 256, rng)
            for k, v in ps.items():
                bundle[f"{name}__e{est}__{k}"] = v
            bundle[f"{name}__e{est}__fb24x24x4"] = ref.render(24, 24, 4, est, seed=SEED)
    np.savez_compressed(os.path.join(HERE, "samples_alt.npz"), **bundle)
    print("wrote", os.path.join(HERE, "samples_alt.npz"))


def surface_pt():
    """iterativePathTracer (include/shadeMethods.h:104, surface only; estimator 5) on every test
    scene and alternate scene -> samples_e5.npz.  Own RNG seed: the other fixtures stay byte-identical."""
    ref = Reference()
    rng = np.random.default_rng(20261017)
    bundle = {}
    for name, mk in {**EST_SCENES, **ALT_SCENES}.items():
        sc = mk()
        ref.set_scene(sc)
        bundle[f"{name}__scene"] = sc.view(np.uint8)
        ps = per_sample(ref, 5, 256, rng)
        for k, v in ps.items():
            bundle[f"{name}__e5__{k}"] = v
        bundle[f"{name}__e5__fb24x24x4"] = ref.render(24, 24, 4, 5, seed=SEED)
    np.savez_compressed(os.path.join(HERE, "samples_e5.npz"), **bundle)
    print("wrote", os.path.join(HERE, "samples_e5.npz"))


# rayMarching3 cases: (scene, light index, step); sigma_a 0.001, sigma_s 0.0125 as src/rt.cpp:791
MARCH_CASES = [("default", 8, 0.1), ("default", 7, 0.1), ("alt_metal_walls", 7, 0.25), ("alt_open_space", 4, 0.5),
               ("alt_light_near_camera", 2, 0.5)]


def ray_marching():
    """rayMarching3 (include/rayMarchingMethods.h:330, estimator 6) -> samples_e6.npz."""
    ref = Reference()
    rng = np.random.default_rng(20261018)
    scenes = {**EST_SCENES, **ALT_SCENES}
    bundle = {}
    for name, light, step in MARCH_CASES:
        sc = scenes[name]()
        ref.set_scene(sc)
        key = f"{name}_l{light}"
        bundle[f"{key}__scene"] = sc.view(np.uint8)
        bundle[f"{key}__march"] = np.array([step, light])
        ref.L.ref_set_march(step, light)
        xs, ys, si = rng.integers(0, W, 96), rng.integers(0, H, 96), rng.integers(0, 1 << 20, 96)
        s0 = np.array([stream_state(SEED, int((H - y - 1) * W + x), int(i)) for x, y, i in zip(xs, ys, si)],
                      dtype=np.uint64)
        rays = np.zeros((96, 6))
        s1 = np.zeros(96, dtype=np.uint64)
        for k in range(96):
            s1[k] = ref.prim("camera_ray")(W, H, int(xs[k]), int(ys[k]), int(s0[k]), rays[k].ctypes.data)
        out, s2 = ref.trace(6, rays, s1, 0.001, 0.0125, march_step=step, march_light=light)
        bundle.update({f"{key}__e6__ray": rays, f"{key}__e6__state1": s1, f"{key}__e6__L": out,
                       f"{key}__e6__state2": s2})
        bundle[f"{key}__e6__fb24x24x2"] = ref.render(24, 24, 2, 6, 0.001, 0.0125, seed=SEED, march_step=step,
                                                     march_light=light)
    np.savez_compressed(os.path.join(HERE, "samples_e6.npz"), **bundle)
    print("wrote", os.path.join(HERE, "samples_e6.npz"))


# rayMarching2 / rayMarchingGlobal / rayMarching cases: (estimator, scene, light index, step or segments);
# sigma_a 0.001, sigma_s 0.0125 as src/rt.cpp:791.  rayMarchingGlobal and rayMarching sample the
# hard-coded sphere 5 (include/rayMarchingMethods.h:64,153): the r = 12 area light of alt_area_light,
# the metal sphere of the default scene.  ("default", 0): rayMarching2's miss id 0 counts as the light.
E789_CASES = [(7, "default", 7, 0.5), (7, "default", 0, 1.0), (7, "alt_area_light", 5, 0.5), (7, "mat3", 9, 0.75),
              (8, "alt_area_light", 0, 6.0), (8, "alt_area_light", 0, 2.5), (8, "default", 0, 4.0),
              (9, "alt_area_light", 0, 10.0), (9, "alt_area_light", 0, 3.5), (9, "default", 0, 10.0)]


def ray_marching_789():
    """rayMarching2 (:262, estimator 7), rayMarchingGlobal (:106, estimator 8), rayMarching (:34,
    estimator 9) of include/rayMarchingMethods.h, plus known answers for punctualVolumetric (:12) and
    rayMarching's out-parameters -> samples_e789.npz.  Own RNG seed."""
    ref = Reference()
    rng = np.random.default_rng(20261019)
    scenes = {**EST_SCENES, **ALT_SCENES}
    bundle = {}
    for est, name, light, step in E789_CASES:
        sc = scenes[name]()
        ref.set_scene(sc)
        key = f"e{est}_{name}_l{light}_s{step}"
        bundle[f"{key}__scene"] = sc.view(np.uint8)
        bundle[f"{key}__march"] = np.array([est, step, light])
        n = 96
        xs, ys, si = rng.integers(0, W, n), rng.integers(0, H, n), rng.integers(0, 1 << 20, n)
        s0 = np.array([stream_state(SEED, int((H - y - 1) * W + x), int(i)) for x, y, i in zip(xs, ys, si)],
                      dtype=np.uint64)
        rays = np.zeros((n, 6))
        s1 = np.zeros(n, dtype=np.uint64)
        for k in range(n):
            s1[k] = ref.prim("camera_ray")(W, H, int(xs[k]), int(ys[k]), int(s0[k]), rays[k].ctypes.data)
        out, s2 = ref.trace(est, rays, s1, 0.001, 0.0125, march_step=step, march_light=light)
        bundle.update({f"{key}__ray": rays, f"{key}__state1": s1, f"{key}__L": out, f"{key}__state2": s2})
        bundle[f"{key}__fb16x16x2"] = ref.render(16, 16, 2, est, 0.001, 0.0125, seed=SEED, march_step=step,
                                                 march_light=light)
    # punctualVolumetric(idsource, x, phase, sigma_t, sigma_s): every emitter of three scenes
    for name in ("default", "mat3", "point_lights"):
        sc = scenes[name]()
        ref.set_scene(sc)
        lights = [i for i in range(len(sc)) if sc[i]["radiance"][0] > 0 or sc[i]["radiance"][1] > 0]
        m = 64 * len(lights)
        ids = np.repeat(np.array(lights, dtype=np.int64), 64)
        xp = np.column_stack([rng.uniform(-48, 48, m), rng.uniform(-40, 40, m), rng.uniform(-80, 100, m)])
        out = np.zeros((m, 3))
        for k in range(m):
            ref.prim("punctual_volumetric")(int(ids[k]), np.ascontiguousarray(xp[k]).ctypes.data, 1 / (4 * np.pi),
                                            0.0135, 0.0125, out[k].ctypes.data)
        bundle.update({f"pv_{name}__scene": sc.view(np.uint8), f"pv_{name}__id": ids, f"pv_{name}__x": xp,
                       f"pv_{name}__out": out})
    # rayMarching's x_new / idsource out-parameters (camera rays of alt_area_light; misses keep the inputs)
    sc = scenes["alt_area_light"]()
    ref.set_scene(sc)
    n = 64
    rays = np.zeros((n, 6))
    s1 = np.zeros(n, dtype=np.uint64)
    for k in range(n):
        x, y = int(rng.integers(0, W)), int(rng.integers(0, H))
        s1[k] = ref.prim("camera_ray")(W, H, x, y, stream_state(SEED, (H - y - 1) * W + x, k), rays[k].ctypes.data)
    rays[::8, 3:6] = (0.0, 1.0, 0.0)  # some rays straight up: alt_area_light has no ceiling (misses)
    out = np.zeros((n, 6))
    ids = np.full(n, -1, dtype=np.int32)
    s2 = np.zeros(n, dtype=np.uint64)
    xin = np.array([1.5, -2.5, 3.25])
    for k in range(n):
        idk = ctypes.c_int(-1)
        s2[k] = ref.prim("ray_marching_explicit")(rays[k].ctypes.data, 0.0135, 0.0125, 7.0, int(s1[k]),
                                                  xin.ctypes.data, ctypes.byref(idk), out[k].ctypes.data)
        ids[k] = idk.value
    bundle.update({"rmx__ray": rays, "rmx__state1": s1, "rmx__out": out, "rmx__id": ids, "rmx__state2": s2,
                   "rmx__xin": xin})
    np.savez_compressed(os.path.join(HERE, "samples_e789.npz"), **bundle)
    print("wrote", os.path.join(HERE, "samples_e789.npz"))


if __name__ == "__main__":
    if sys.argv[1:] == ["--estimators-234"]:
        estimators_234()
    elif sys.argv[1:] == ["--alt-scenes"]:
        alt_scenes()
    elif sys.argv[1:] == ["--surface-pt"]:
        surface_pt()
    elif sys.argv[1:] == ["--ray-marching"]:
        ray_marching()
    elif sys.argv[1:] == ["--ray-marching-789"]:
        ray_marching_789()
    else:
        main()
        estimators_234()
        alt_scenes()
        surface_pt()
        ray_marching()
        ray_marching_789()
