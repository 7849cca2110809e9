"""MI355X-native volumetric path tracer: the per-pixel radiance loop of
gabo99cas/minimal_volumetric_path_tracer (src/rt.cpp, include/vptShadeMethods.h) as HIP kernels
for gfx950 behind a C ABI (include/vpt.h, libvpt.so).  See DESIGN.md."""
from ._lib import (EXPLICIT_EQUIANGULAR, EXPLICIT_FREE, FB_F32, FB_F64, FREE_FLIGHT, IMPLICIT_FREE, MIS_EQUIANGULAR,
                   RAY_DTYPE, RAY_MARCHING, RAY_MARCHING_EXPLICIT, RAY_MARCHING_GLOBAL, RAY_MARCHING_SA, SPHERE_DTYPE,
                   SURFACE_PT, VPTError, build_id, lib)
from .tracer import (
    MultiTracer,
    Ray,
    RenderConfig,
    Sphere,
    Tracer,
    default_scene,
    encode_ppm,
    render_multi,
    scene,
    stream_state,
    write_ppm,
)

__all__ = [
    "FB_F32", "FB_F64", "FREE_FLIGHT", "MIS_EQUIANGULAR", "EXPLICIT_FREE", "IMPLICIT_FREE", "EXPLICIT_EQUIANGULAR", "SURFACE_PT", "RAY_MARCHING",
    "RAY_MARCHING_SA", "RAY_MARCHING_GLOBAL", "RAY_MARCHING_EXPLICIT", "RAY_DTYPE", "SPHERE_DTYPE", "VPTError", "build_id", "lib",
    "MultiTracer", "render_multi", "Ray", "RenderConfig", "Sphere", "Tracer", "default_scene", "encode_ppm", "scene", "stream_state", "write_ppm",
]
