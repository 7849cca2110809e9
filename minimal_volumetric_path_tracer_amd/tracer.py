"""Host-side mirror of the reference's interface for the volumetric radiance loop.

Reference (gabo99cas/minimal_volumetric_path_tracer):
  * scene: ``std::vector<Sphere> spheres`` (include/Sphere.h:49, include/Sphere.cpp:7-107) with
    ``Sphere(r, p, c, radiance, material, eta, kappa, alpha)`` (include/Sphere.h:23);
  * per-sample estimators ``iterativeVPTracerFree(ray, sigma_a, sigma_s)``
    (include/vptShadeMethods.h:1263, the one ``main`` calls), ``MISVPTTracerRecursive(ray, sigma_a,
    sigma_s, depth)`` (:1345), ``explicitVPTracerRecursiveFree`` (:1153),
    ``implicitVPTracerRecursiveFree`` (:940) and ``explicitVPTracerRecursive`` (:1014), returning a Color;
  * ``main`` (src/rt.cpp:744-830): camera, pixel loop, average, clamp, ``image.ppm``.

Here the same names take batches and run through libvpt.so (HIP, gfx950).  Argument meaning is
the reference's; its undefined behaviour (uninitialised argv, >4 emitters, unchecked fopen)
becomes an exception.
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, byref, c_int, c_uint64, c_void_p
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (EXPLICIT_EQUIANGULAR, EXPLICIT_FREE, FB_F32, FB_F64, FREE_FLIGHT, IMPLICIT_FREE, MIS_EQUIANGULAR,
                   RAY_DTYPE, RAY_MARCHING, RAY_MARCHING_EXPLICIT, RAY_MARCHING_GLOBAL, RAY_MARCHING_SA, SPHERE_DTYPE,
                   SURFACE_PT, check, lib)

ESTIMATORS = {"ff": FREE_FLIGHT, "free_flight": FREE_FLIGHT, "mis": MIS_EQUIANGULAR, "mis_equiangular": MIS_EQUIANGULAR,
              "explicit_free": EXPLICIT_FREE, "implicit_free": IMPLICIT_FREE, "explicit": EXPLICIT_EQUIANGULAR,
              "explicit_equiangular": EXPLICIT_EQUIANGULAR, "surface_pt": SURFACE_PT, "path_tracer": SURFACE_PT,
              "ray_marching": RAY_MARCHING, "ray_marching_sa": RAY_MARCHING_SA, "ray_marching_global": RAY_MARCHING_GLOBAL,
              "ray_marching_explicit": RAY_MARCHING_EXPLICIT}


def Sphere(r, p, c=(0, 0, 0), radiance=(0, 0, 0), material=0, eta=(0, 0, 0), kappa=(0, 0, 0), alpha=0.0) -> np.ndarray:
    """One reference Sphere record (include/Sphere.h:23 argument order) as a SPHERE_DTYPE scalar array."""
    s = np.zeros(1, dtype=SPHERE_DTYPE)
    s["r"], s["p"], s["c"], s["radiance"] = r, p, c, radiance
    s["material"], s["eta"], s["kappa"], s["alpha"] = material, eta, kappa, alpha
    return s


def scene(*spheres: np.ndarray) -> np.ndarray:
    return np.concatenate(spheres).astype(SPHERE_DTYPE)


def default_scene() -> np.ndarray:
    """The reference scene, include/Sphere.cpp:11-22 (10 spheres)."""
    n = lib().vpt_default_scene(None, 0)
    out = np.zeros(n, dtype=SPHERE_DTYPE)
    lib().vpt_default_scene(out.ctypes.data, n)
    return out


def Ray(o: Sequence[float], d: Sequence[float]) -> np.ndarray:
    r = np.zeros(1, dtype=RAY_DTYPE)
    r["o"], r["d"] = o, d
    return r


def stream_state(seed: int, pixel_idx: int, sample: int) -> int:
    """erand48 start state of one camera sample (csrc/vpt_rng.h)."""
    return int(lib().vpt_stream_state(seed, pixel_idx, sample))


@dataclass
class RenderConfig:
    width: int = 1024
    height: int = 768
    spp: int = 16
    estimator: str = "ff"
    sigma_a: float = 0.001
    sigma_s: float = 0.009
    hg_g: float = 0.0
    max_depth: int = 0
    seed: int = 0x5EED0001
    fp64: bool = False
    band_rows: int = 0          # 0 = whole image
    band_stride: int = 1
    band_offset: int = 0
    chunk_spp: int = 0          # 0 = auto (min(spp, 32), the last 64 samples tapered); 1 or >= spp = the reference's sequential sum
    march_step: float = 0.1     # ray marching: step (rayMarching3 / rayMarching2, src/rt.cpp:791) or segments
                                # (rayMarchingGlobal / rayMarching)
    march_light: int = 7        # rayMarching3 / rayMarching2: light sphere index (src/rt.cpp:791)

    def params(self) -> _lib.vpt_params:
        p = _lib.vpt_params()
        lib().vpt_default_params(byref(p))
        p.width, p.height, p.spp = self.width, self.height, self.spp
        p.fb_format = FB_F64 if self.fp64 else FB_F32
        p.medium.sigma_a, p.medium.sigma_s = self.sigma_a, self.sigma_s
        p.medium.hg_g, p.medium.max_depth = self.hg_g, self.max_depth
        p.medium.estimator = ESTIMATORS[self.estimator] if isinstance(self.estimator, str) else int(self.estimator)
        p.medium.march_step, p.medium.march_light = self.march_step, self.march_light
        p.seed = self.seed
        p.band_rows = self.band_rows if self.band_rows > 0 else self.height
        p.band_stride, p.band_offset = self.band_stride, self.band_offset
        p.chunk_spp = self.chunk_spp
        return p

    def shard_rows(self) -> int:
        return int(lib().vpt_shard_rows(byref(self.params())))

    def medium(self) -> _lib.vpt_medium:
        return self.params().medium


class Tracer:
    """One GPU context with one scene (replaces the reference's global ``spheres``)."""

    def __init__(self, device: int = 0, spheres: Optional[np.ndarray] = None):
        h = c_void_p()
        check(lib().vpt_context_create(device, byref(h)))
        self._ctx = h
        self.device = device
        self.set_scene(default_scene() if spheres is None else spheres)

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            lib().vpt_context_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, spheres: np.ndarray) -> None:
        s = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
        check(lib().vpt_set_scene(self._ctx, s.ctypes.data, len(s)))
        self.spheres = s

    # ---- main()'s pixel loop (src/rt.cpp:767-805) ----
    def render(self, cfg: Optional[RenderConfig] = None, **kw) -> np.ndarray:
        """Renders on the GPU; returns (shard_rows, width, 3) in file order (row 0 = top), the
        per-pixel average before the clamp of src/rt.cpp:803."""
        cfg = cfg or RenderConfig(**kw)
        p = cfg.params()
        rows = int(lib().vpt_shard_rows(byref(p)))
        out = np.zeros((max(rows, 1), cfg.width, 3), dtype=np.float64 if cfg.fp64 else np.float32)
        check(lib().vpt_render(self._ctx, byref(p), out.ctypes.data))  # validates even an empty shard
        return out[:rows]

    def render_device(self, cfg: RenderConfig, out_ptr: int, stream: int = 0) -> None:
        """Enqueues a render into a device buffer (e.g. torch tensor .data_ptr()) on `stream`."""
        p = cfg.params()
        check(lib().vpt_render_device(self._ctx, byref(p), c_void_p(out_ptr), c_void_p(stream)))

    def count_work(self, cfg: RenderConfig) -> tuple[int, int]:
        """(ray-sphere tests, estimator iterations) of the reference algorithm for this render."""
        t, i = c_uint64(), c_uint64()
        check(lib().vpt_count_work(self._ctx, byref(cfg.params()), byref(t), byref(i)))
        return int(t.value), int(i.value)

    # ---- the per-sample estimators, batched ----
    def trace(self, estimator, rays: np.ndarray, states: np.ndarray, sigma_a=0.001, sigma_s=0.009, hg_g=0.0,
              max_depth=0, march_step=0.1, march_light=7) -> tuple[np.ndarray, np.ndarray]:
        m = _lib.vpt_medium(sigma_a, sigma_s, hg_g, max_depth,
                            ESTIMATORS[estimator] if isinstance(estimator, str) else int(estimator), march_step,
                            march_light)
        r = np.ascontiguousarray(rays, dtype=RAY_DTYPE)
        s = np.ascontiguousarray(states, dtype=np.uint64)
        if len(r) != len(s):
            raise ValueError("rays and states must have the same length")
        out = np.zeros((len(r), 3), dtype=np.float64)
        st = np.zeros(len(r), dtype=np.uint64)
        check(lib().vpt_trace_batch(self._ctx, byref(m), r.ctypes.data, s.ctypes.data, len(r), out.ctypes.data,
                                    st.ctypes.data))
        return out, st

    def iterativeVPTracerFree(self, rays, states, sigma_a=0.001, sigma_s=0.009, **kw):
        """Batched include/vptShadeMethods.h:1263."""
        return self.trace("ff", rays, states, sigma_a, sigma_s, **kw)

    def MISVPTTracerRecursive(self, rays, states, sigma_a=0.001, sigma_s=0.009, **kw):
        """Batched include/vptShadeMethods.h:1345 (depth 0)."""
        return self.trace("mis", rays, states, sigma_a, sigma_s, **kw)

    def explicitVPTracerRecursiveFree(self, rays, states, sigma_a=0.001, sigma_s=0.009, **kw):
        """Batched include/vptShadeMethods.h:1153 (depth 0)."""
        return self.trace("explicit_free", rays, states, sigma_a, sigma_s, **kw)

    def implicitVPTracerRecursiveFree(self, rays, states, sigma_a=0.001, sigma_s=0.009, **kw):
        """Batched include/vptShadeMethods.h:940."""
        return self.trace("implicit_free", rays, states, sigma_a, sigma_s, **kw)

    def explicitVPTracerRecursive(self, rays, states, sigma_a=0.001, sigma_s=0.009, **kw):
        """Batched include/vptShadeMethods.h:1014 (depth 0)."""
        return self.trace("explicit", rays, states, sigma_a, sigma_s, **kw)

    def iterativePathTracer(self, rays, states):
        """Batched include/shadeMethods.h:104 (surface only: no medium arguments)."""
        return self.trace("surface_pt", rays, states)

    def rayMarching3(self, rays, states, sigma_a, sigma_s, step, idsource):
        """Batched include/rayMarchingMethods.h:330 (src/rt.cpp:791 passes 0.001, 0.0125, 0.1, 7)."""
        return self.trace("ray_marching", rays, states, sigma_a, sigma_s, march_step=step, march_light=idsource)

    def rayMarching2(self, rays, states, sigma_a, sigma_s, step, idsource):
        """Batched include/rayMarchingMethods.h:262."""
        return self.trace("ray_marching_sa", rays, states, sigma_a, sigma_s, march_step=step, march_light=idsource)

    def rayMarchingGlobal(self, rays, states, sigma_a, sigma_s, segmentos):
        """Batched include/rayMarchingMethods.h:106 (samples the hard-coded sphere 5)."""
        return self.trace("ray_marching_global", rays, states, sigma_a, sigma_s, march_step=segmentos)

    def rayMarching(self, rays, states, sigma_t, sigma_s, steps, x_new=None, idsource=None):
        """Batched include/rayMarchingMethods.h:34 with its reference parameters: returns
        (Color, x_new, idsource, end states); x_new / idsource are kept on a miss (inputs default
        to 0 / -1)."""
        r = np.ascontiguousarray(rays, dtype=RAY_DTYPE)
        s = np.ascontiguousarray(states, dtype=np.uint64)
        if len(r) != len(s):
            raise ValueError("rays and states must have the same length")
        xn = np.zeros((len(r), 3))
        if x_new is not None:
            xn[:] = x_new
        ids = np.full(len(r), -1, dtype=np.int32)
        if idsource is not None:
            ids[:] = idsource
        out = np.zeros((len(r), 3))
        st = np.zeros(len(r), dtype=np.uint64)
        check(lib().vpt_ray_marching_batch(self._ctx, float(sigma_t), float(sigma_s), float(steps), r.ctypes.data,
                                           s.ctypes.data, len(r), out.ctypes.data, xn.ctypes.data, ids.ctypes.data,
                                           st.ctypes.data))
        return out, xn, ids, st

    def punctualVolumetric(self, idsource: int, x: np.ndarray, phase: float, sigma_t: float, sigma_s: float) -> np.ndarray:
        """include/rayMarchingMethods.h:12 at every point of x (n x 3) -> (n x 3) Colors."""
        xs = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float64)
        out = np.zeros_like(xs)
        check(lib().vpt_punctual_volumetric(self._ctx, int(idsource), xs.ctypes.data, len(xs), float(phase),
                                            float(sigma_t), float(sigma_s), out.ctypes.data))
        return out

    def math_probe(self, fn: int, x: np.ndarray, y: Optional[np.ndarray] = None) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, dtype=np.float64)
        out = np.zeros_like(x)
        check(lib().vpt_math_probe(self._ctx, fn, x.ctypes.data, y.ctypes.data, out.ctypes.data, len(x)))
        return out

    def hg_phase(self, g: float, din, states: np.ndarray, wl: np.ndarray):
        """HG phase extension on the GPU (vpt_phase_probe): (directions sampled around din, end states,
        phase values toward the rows of wl)."""
        d = np.ascontiguousarray(din, dtype=np.float64)
        s = np.ascontiguousarray(states, dtype=np.uint64)
        w = np.ascontiguousarray(wl, dtype=np.float64).reshape(-1, 3)
        dirs = np.zeros((len(s), 3))
        so = np.zeros(len(s), dtype=np.uint64)
        vals = np.zeros(len(w))
        check(lib().vpt_phase_probe(self._ctx, float(g), d.ctypes.data, s.ctypes.data, len(s), dirs.ctypes.data,
                                    so.ctypes.data, w.ctypes.data, len(w), vals.ctypes.data))
        return dirs, so, vals


class MultiTracer:
    """Devices 0 .. n_gpus-1 of THIS process rendering one image together (vpt_multi_*, include/vpt.h):
    interleaved row bands per device, strips gathered to device 0 over RCCL.  Bit-identical to
    Tracer.render for any n_gpus."""

    def __init__(self, n_gpus: int, spheres: Optional[np.ndarray] = None, shared_device: bool = False):
        """shared_device (tests): n_gpus logical ranks on device 0, their strips copied on the device
        instead of sent over RCCL (vpt_debug_multi_create_shared) -- the n > 1 path on a one-GPU box"""
        h = c_void_p()
        if shared_device:
            f = lib().vpt_debug_multi_create_shared
            f.restype, f.argtypes = c_int, [c_int, POINTER(c_void_p)]
            check(f(n_gpus, byref(h)))
        else:
            check(lib().vpt_multi_create(n_gpus, byref(h)))
        self._m = h
        self.n_gpus = n_gpus
        s = np.ascontiguousarray(default_scene() if spheres is None else spheres, dtype=SPHERE_DTYPE)
        check(lib().vpt_multi_set_scene(self._m, s.ctypes.data, len(s)))
        self.spheres = s

    def render(self, cfg: Optional[RenderConfig] = None, **kw) -> np.ndarray:
        """(height, width, 3), file order; cfg.band_rows (when it cuts the image) is the band size."""
        cfg = cfg or RenderConfig(**kw)
        p = cfg.params()
        out = np.zeros((cfg.height, cfg.width, 3), dtype=np.float64 if cfg.fp64 else np.float32)
        check(lib().vpt_multi_render(self._m, byref(p), out.ctypes.data))
        return out

    def close(self) -> None:
        if getattr(self, "_m", None):
            lib().vpt_multi_destroy(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_multi(n_gpus: int, cfg: Optional[RenderConfig] = None, spheres: Optional[np.ndarray] = None,
                 **kw) -> np.ndarray:
    """One-shot vpt_render_multi: the image of `cfg` on devices 0 .. n_gpus-1."""
    cfg = cfg or RenderConfig(**kw)
    s = np.ascontiguousarray(default_scene() if spheres is None else spheres, dtype=SPHERE_DTYPE)
    p = cfg.params()
    out = np.zeros((cfg.height, cfg.width, 3), dtype=np.float64 if cfg.fp64 else np.float32)
    check(lib().vpt_render_multi(s.ctypes.data, len(s), byref(p), n_gpus, out.ctypes.data))
    return out


# ---- output (src/rt.cpp:812-820) ----
def _fb(rgb: np.ndarray) -> tuple[np.ndarray, int, int, int]:
    a = np.ascontiguousarray(rgb)
    if a.dtype == np.float32:
        fmt = FB_F32
    elif a.dtype == np.float64:
        fmt = FB_F64
    else:
        a, fmt = np.ascontiguousarray(a, dtype=np.float64), FB_F64
    if a.ndim != 3 or a.shape[2] != 3:
        raise ValueError("framebuffer must be (height, width, 3)")
    return a, fmt, a.shape[1], a.shape[0]


def encode_ppm(rgb: np.ndarray) -> bytes:
    a, fmt, w, h = _fb(rgb)
    n = lib().vpt_encode_ppm(a.ctypes.data, fmt, w, h, None, 0)
    if n < 0:
        check(int(n))
    buf = ctypes.create_string_buffer(int(n))
    m = lib().vpt_encode_ppm(a.ctypes.data, fmt, w, h, buf, n)
    if m != n:
        check(int(m) if m < 0 else _lib.VPT_E_INVALID)
    return buf.raw


def write_ppm(path: str, rgb: np.ndarray) -> None:
    a, fmt, w, h = _fb(rgb)
    check(lib().vpt_write_ppm(path.encode(), a.ctypes.data, fmt, w, h))
