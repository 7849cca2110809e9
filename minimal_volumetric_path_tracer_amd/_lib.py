"""ctypes binding of libvpt.so (the C ABI of include/vpt.h).

This is the whole product boundary: every render goes through the HIP kernels in
csrc/vpt_kernels.hip.  There is no CPU fallback -- if the shared library is missing or no GPU
is visible, calls raise instead of computing anything another way.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_uint64, c_void_p

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# VPT_LIB: path of an alternative build of the same ABI (A/B timing of kernel variants)
LIB_PATH = os.environ.get("VPT_LIB") or os.path.join(PKG_DIR, "libvpt.so")
CLI_PATH = os.path.join(PKG_DIR, "vpt")

VPT_OK = 0
VPT_E_INVALID, VPT_E_TOO_MANY, VPT_E_NO_EMITTER, VPT_E_UNSUPPORTED, VPT_E_HIP, VPT_E_IO, VPT_E_INTERNAL = \
    -1, -2, -3, -4, -5, -6, -7
VPT_MAX_SPHERES = 64
FREE_FLIGHT, MIS_EQUIANGULAR, EXPLICIT_FREE, IMPLICIT_FREE, EXPLICIT_EQUIANGULAR, SURFACE_PT, RAY_MARCHING = 0, 1, 2, 3, 4, 5, 6  # vpt_estimator
RAY_MARCHING_SA, RAY_MARCHING_GLOBAL, RAY_MARCHING_EXPLICIT = 7, 8, 9
FB_F32, FB_F64 = 0, 1

# numpy view of vpt_sphere == reference Sphere (include/Sphere.h:12-21), 144 bytes
SPHERE_DTYPE = np.dtype(
    {
        "names": ["r", "p", "c", "radiance", "material", "reserved_", "eta", "kappa", "alpha"],
        "formats": ["<f8", ("<f8", 3), ("<f8", 3), ("<f8", 3), "<i4", "<i4", ("<f8", 3), ("<f8", 3), "<f8"],
        "offsets": [0, 8, 32, 56, 80, 84, 88, 112, 136],
        "itemsize": 144,
    }
)
RAY_DTYPE = np.dtype([("o", "<f8", 3), ("d", "<f8", 3)])


class vpt_ray(ctypes.Structure):
    _fields_ = [("o", c_double * 3), ("d", c_double * 3)]


class vpt_medium(ctypes.Structure):
    _fields_ = [
        ("sigma_a", c_double),
        ("sigma_s", c_double),
        ("hg_g", c_double),
        ("max_depth", c_int32),
        ("estimator", c_int32),
        ("march_step", c_double),
        ("march_light", c_int32),
        ("reserved_", c_int32),
    ]


class vpt_params(ctypes.Structure):
    _fields_ = [
        ("width", c_int32),
        ("height", c_int32),
        ("spp", c_int32),
        ("fb_format", c_int32),
        ("medium", vpt_medium),
        ("seed", c_uint64),
        ("camera", vpt_ray),
        ("fov_scale", c_double),
        ("band_rows", c_int32),
        ("band_stride", c_int32),
        ("band_offset", c_int32),
        ("chunk_spp", c_int32),
    ]


class VPTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libvpt error {code}: {msg}")
        self.code = code


_lib = None

# (name, restype, argtypes) -- exactly the functions include/vpt.h declares
PROTOTYPES = [
    ("vpt_default_params", None, [POINTER(vpt_params)]),
    ("vpt_default_scene", c_int, [c_void_p, c_int]),
    ("vpt_shard_rows", c_int, [POINTER(vpt_params)]),
    ("vpt_context_create", c_int, [c_int, POINTER(c_void_p)]),
    ("vpt_context_destroy", None, [c_void_p]),
    ("vpt_set_scene", c_int, [c_void_p, c_void_p, c_int]),
    ("vpt_render_device", c_int, [c_void_p, POINTER(vpt_params), c_void_p, c_void_p]),
    ("vpt_render", c_int, [c_void_p, POINTER(vpt_params), c_void_p]),
    ("vpt_multi_create", c_int, [c_int, POINTER(c_void_p)]),
    ("vpt_multi_set_scene", c_int, [c_void_p, c_void_p, c_int]),
    ("vpt_multi_render", c_int, [c_void_p, POINTER(vpt_params), c_void_p]),
    ("vpt_multi_destroy", None, [c_void_p]),
    ("vpt_render_multi", c_int, [c_void_p, c_int, POINTER(vpt_params), c_int, c_void_p]),
    ("vpt_trace_batch", c_int, [c_void_p, POINTER(vpt_medium), c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    ("vpt_punctual_volumetric", c_int, [c_void_p, c_int, c_void_p, c_int, c_double, c_double, c_double, c_void_p]),
    ("vpt_ray_marching_batch", c_int, [c_void_p, c_double, c_double, c_double, c_void_p, c_void_p, c_int, c_void_p,
                                       c_void_p, c_void_p, c_void_p]),
    ("vpt_count_work", c_int, [c_void_p, POINTER(vpt_params), POINTER(c_uint64), POINTER(c_uint64)]),
    ("vpt_stream_state", c_uint64, [c_uint64, c_uint64, c_uint64]),
    ("vpt_math_probe", c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int]),
    ("vpt_phase_probe", c_int, [c_void_p, c_double, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                c_void_p]),
    ("vpt_write_ppm", c_int, [c_char_p, c_void_p, c_int, c_int, c_int]),
    ("vpt_encode_ppm", c_int64, [c_void_p, c_int, c_int, c_int, c_void_p, c_int64]),
    ("vpt_last_error", c_char_p, []),
    ("vpt_abi_version", c_int, []),
    ("vpt_build_id", c_char_p, []),
]


def lib() -> ctypes.CDLL:
    """The loaded libvpt.so; raises if it was not built (no fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or `make -C minimal_volumetric_path_tracer_amd/csrc`); there is no CPU fallback"
            )
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in PROTOTYPES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def build_id() -> str:
    """The loaded library's build id (sources + flags hash, scripts/build_id.py)."""
    return lib().vpt_build_id().decode()


def check(rc: int) -> None:
    if rc != VPT_OK:
        msg = lib().vpt_last_error()
        raise VPTError(rc, msg.decode() if msg else "")
