"""TEST INFRASTRUCTURE ONLY -- ctypes access to the parity oracle (oracle/README in DESIGN.md).

Loaders for
  * liboracle.so      C restatement, libm transcendentals  (pinned to the reference itself),
  * liboracle_vm.so   the same restatement with the build's portable FP64 math (= the kernel's arithmetic),
  * _ref/libvpt_ref.so  the reference's own functions compiled in place (only where /root/reference was
                        available at build time; the built .so travels with the repo).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, byref, c_double, c_int, c_int32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SPHERE_BYTES = 144


class Medium(ctypes.Structure):
    _fields_ = [("sigma_a", c_double), ("sigma_s", c_double), ("hg_g", c_double), ("max_depth", c_int32),
                ("estimator", c_int32), ("march_step", c_double), ("march_light", c_int32), ("reserved_", c_int32)]


class Counters(ctypes.Structure):
    _fields_ = [("tests", c_uint64), ("iterations", c_uint64), ("surface", c_uint64), ("medium", c_uint64)]


_P = c_void_p
_U = c_uint64
_D = c_double
_I = c_int

_PRIMS = {
    # name: (restype, argtypes) -- identical for orc_* and ref_*
    "sphere_intersect": (_D, [_I, _P]),
    "intersect": (_I, [_P, _P, _P]),
    "visibility": (_I, [_P, _P]),
    "transmitance": (_D, [_P, _P, _D]),
    "coordinate_system": (None, [_P, _P, _P]),
    "solid_angle_dir": (_U, [_P, _D, _U, _P]),
    "cosine_hemispheric": (_U, [_P, _U, _P]),
    "isotropic_phase": (_U, [_U, _P]),
    "vector_facet": (_U, [_D, _U, _P]),
    "fresnel": (None, [_D, _P, _P, _P]),
    "fr_microfacet": (None, [_P, _P, _P, _P, _P, _D, _P, _P]),
    "microfacet_prob": (_D, [_P, _P, _D, _P]),
    "bdsf": (_U, [_P, _P, _I, _U, _P, _P, _P]),
    "plight": (None, [_I, _P, _P, _P, _P, _P, _D, _P]),
    "misv2": (_U, [_I, _P, _P, _P, _D, _D, _U, _P]),
    "free_single_scattering": (_U, [_P, _I, _D, _D, _U, _P]),
    "single_scattering": (_U, [_P, _I, _D, _D, _D, _D, _U, _P]),
    "equiangular_params2": (_U, [_I, _D, _P, _P, _U]),
    "equiangular_prob": (_D, [_D, _D, _D, _D]),
    "camera_ray": (_U, [_I, _I, _I, _I, _U, _P]),
    "to_display": (_I, [_D]),
    "punctual_volumetric": (None, [_I, _P, _D, _D, _D, _P]),
    "ray_marching_explicit": (_U, [_P, _D, _D, _D, _U, _P, _P, _P]),
}


def _bind(L: ctypes.CDLL, prefix: str) -> ctypes.CDLL:
    for name, (res, args) in _PRIMS.items():
        fn = getattr(L, f"{prefix}_{name}")
        fn.restype, fn.argtypes = res, args
    return L


def default_chunk(spp: int) -> int:
    """samples per chunk the GPU uses when vpt_params.chunk_spp == 0 (vpt_auto_chunk, csrc/vpt_chunks.h)"""
    return min(spp, max(32, -(-spp // 128)))


class Oracle:
    """liboracle.so (portable=False) or liboracle_vm.so (portable=True)."""

    def __init__(self, portable: bool = False):
        path = os.path.join(HERE, "liboracle_vm.so" if portable else "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built (make -C oracle oracle)")
        L = ctypes.CDLL(path)
        _bind(L, "orc")
        L.orc_set_scene.restype, L.orc_set_scene.argtypes = _I, [_P, _I]
        L.orc_trace.restype = _U
        L.orc_trace.argtypes = [_P, _U, POINTER(Medium), _P, POINTER(Counters)]
        L.orc_render.restype = None
        L.orc_render.argtypes = [_I, _I, _I, POINTER(Medium), _U, _I, _I, _P, _I, POINTER(Counters)]
        L.orc_render_chunked.restype = None
        L.orc_render_chunked.argtypes = [_I, _I, _I, _I, POINTER(Medium), _U, _I, _I, _P, _I, POINTER(Counters)]
        L.orc_render_layout.restype = None
        L.orc_render_layout.argtypes = [_I, _I, _I, _I, _I, POINTER(Medium), _U, _I, _I, _P, _I, POINTER(Counters)]
        L.orc_write_ppm.restype, L.orc_write_ppm.argtypes = _I, [ctypes.c_char_p, _P, _I, _I]
        L.orc_stream_state_c.restype, L.orc_stream_state_c.argtypes = _U, [_U, _U, _U]
        L.orc_is_portable_math.restype = _I
        L.orc_math_n.restype, L.orc_math_n.argtypes = None, [_I, _P, _P, _P, _I]
        L.orc_hg_phase_sample.restype, L.orc_hg_phase_sample.argtypes = _U, [_D, _P, _U, _P]
        L.orc_hg_phase_value.restype, L.orc_hg_phase_value.argtypes = _D, [_D, _P, _P]
        self.L = L
        self.portable = bool(L.orc_is_portable_math())
        self.prefix = "orc"

    def set_scene(self, spheres: np.ndarray) -> None:
        b = np.ascontiguousarray(spheres).view(np.uint8)
        n = len(b) // SPHERE_BYTES
        if self.L.orc_set_scene(b.ctypes.data, n) != 0:
            raise ValueError("oracle: bad scene")

    def hg_phase(self, g: float, din, states: np.ndarray, wl: np.ndarray):
        """HG extension (phase_sample / phase_value): directions sampled around din from each erand48
        state, the end states, and the phase values toward the rows of wl."""
        d = np.ascontiguousarray(din, dtype=np.float64)
        w = np.ascontiguousarray(wl, dtype=np.float64).reshape(-1, 3)
        n = len(states)
        out = np.zeros((n, 3))
        st = np.zeros(n, dtype=np.uint64)
        pv = np.zeros(len(w))
        for i in range(n):
            st[i] = self.L.orc_hg_phase_sample(g, d.ctypes.data, int(states[i]), out[i].ctypes.data)
        for i in range(len(w)):
            pv[i] = self.L.orc_hg_phase_value(g, d.ctypes.data, w[i].ctypes.data)
        return out, st, pv

    def trace(self, estimator: int, rays: np.ndarray, states: np.ndarray, sigma_a=0.001, sigma_s=0.009, hg_g=0.0,
              max_depth=0, counters: bool = False, march_step=0.1, march_light=7):
        m = Medium(sigma_a, sigma_s, hg_g, max_depth, estimator, march_step, march_light)
        r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        out = np.zeros((len(r), 3))
        st = np.zeros(len(r), dtype=np.uint64)
        tot = [0, 0, 0, 0]
        c = Counters()
        for i in range(len(r)):
            st[i] = self.L.orc_trace(r[i].ctypes.data, int(states[i]), byref(m), out[i].ctypes.data,
                                     byref(c) if counters else None)
            if counters:
                tot = [tot[0] + c.tests, tot[1] + c.iterations, tot[2] + c.surface, tot[3] + c.medium]
        return (out, st, tot) if counters else (out, st)

    def render(self, w, h, spp, estimator=0, sigma_a=0.001, sigma_s=0.009, hg_g=0.0, max_depth=0, seed=0x5EED0001,
               y0=0, y1=None, threads=0, counters=False, chunk=None, march_step=0.1, march_light=7):
        """main()'s pixel loop over camera rows [y0, y1); returns (h, w, 3) float64 in file order.
        chunk: samples per partial sum in uniform chunks (spp = the reference's order); None = the
        GPU's default (vpt_params.chunk_spp == 0): chunks of min(spp, 32), the last 32 tapered
        (csrc/vpt_chunks.h)."""
        m = Medium(sigma_a, sigma_s, hg_g, max_depth, estimator, march_step, march_light)
        out = np.zeros((h, w, 3))
        c = Counters()
        taper = 0
        if chunk is None or chunk == 0:
            chunk, taper = default_chunk(spp), 1
        self.L.orc_render_layout(w, h, spp, chunk, taper, byref(m), seed, y0, h if y1 is None else y1,
                                 out.ctypes.data, threads, byref(c))
        return (out, c) if counters else out

    def math(self, fn: int, x: np.ndarray, y=None) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, dtype=np.float64)
        out = np.zeros_like(x)
        self.L.orc_math_n(fn, x.ctypes.data, y.ctypes.data, out.ctypes.data, len(x))
        return out

    def stream_state(self, seed, idx, sample) -> int:
        return int(self.L.orc_stream_state_c(seed, idx, sample))

    def camera_ray(self, w, h, x, y, state):
        r = np.zeros(6)
        s = self.L.orc_camera_ray(w, h, x, y, state, r.ctypes.data)
        return r, int(s)

    def write_ppm(self, path: str, lin: np.ndarray) -> None:
        a = np.ascontiguousarray(lin, dtype=np.float64)
        if self.L.orc_write_ppm(path.encode(), a.ctypes.data, a.shape[1], a.shape[0]) != 0:
            raise OSError(path)

    def prim(self, name):
        return getattr(self.L, f"{self.prefix}_{name}")


class Reference:
    """oracle/_ref/libvpt_ref.so: the reference's own functions (ref_harness.cpp)."""

    PATH = os.path.join(HERE, "_ref", "libvpt_ref.so")

    def __init__(self):
        if not os.path.exists(self.PATH):
            raise FileNotFoundError(self.PATH)
        L = ctypes.CDLL(self.PATH)
        _bind(L, "ref")
        L.ref_default_scene.restype, L.ref_default_scene.argtypes = _I, [_P, _I]
        L.ref_set_scene.restype, L.ref_set_scene.argtypes = None, [_P, _I]
        L.ref_trace.restype, L.ref_trace.argtypes = _U, [_I, _P, _U, _D, _D, _P]
        L.ref_render.restype = None
        L.ref_render.argtypes = [_I, _I, _I, _I, _D, _D, _U, _I, _I, _P, _P]
        L.ref_sizeof_sphere.restype = _I
        L.ref_set_march.restype, L.ref_set_march.argtypes = None, [_D, _I]
        self.L = L
        self.prefix = "ref"

    @staticmethod
    def available() -> bool:
        return os.path.exists(Reference.PATH)

    def default_scene(self) -> np.ndarray:
        n = self.L.ref_default_scene(None, 0)
        b = np.zeros(n * SPHERE_BYTES, dtype=np.uint8)
        self.L.ref_default_scene(b.ctypes.data, n)
        return b

    def set_scene(self, spheres: np.ndarray) -> None:
        b = np.ascontiguousarray(spheres).view(np.uint8)
        self.L.ref_set_scene(b.ctypes.data, len(b) // SPHERE_BYTES)

    def trace(self, estimator, rays, states, sigma_a=0.001, sigma_s=0.009, march_step=0.1, march_light=7):
        self.L.ref_set_march(march_step, march_light)
        r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        out = np.zeros((len(r), 3))
        st = np.zeros(len(r), dtype=np.uint64)
        for i in range(len(r)):
            st[i] = self.L.ref_trace(estimator, r[i].ctypes.data, int(states[i]), sigma_a, sigma_s, out[i].ctypes.data)
        return out, st

    def render(self, w, h, spp, estimator=0, sigma_a=0.001, sigma_s=0.009, seed=0x5EED0001, y0=0, y1=None,
               per_sample=False, march_step=0.1, march_light=7):
        self.L.ref_set_march(march_step, march_light)
        out = np.zeros((h, w, 3))
        ps = np.zeros((h * w * spp, 3)) if per_sample else None
        self.L.ref_render(w, h, spp, estimator, sigma_a, sigma_s, seed, y0, h if y1 is None else y1, out.ctypes.data,
                          ps.ctypes.data if per_sample else None)
        return (out, ps) if per_sample else out

    def prim(self, name):
        return getattr(self.L, f"{self.prefix}_{name}")
