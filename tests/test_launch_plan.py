"""The pool's launch split, on the CPU (vpt_debug_launch_plan: the same units and the same split that
launch_pool applies before enqueueing).  A render whose units exceed 2^26 samples per workgroup is
cut into launches [unit0, unit0 + nunits) in unit order; each unit owns one partial slot, so the cut
changes no value (src/rt.cpp:786-800: every sample of a pixel summed once, in order).  BASELINE
configs[4] -- 4096^2 x 8192 MIS over 8 GPUs -- is the workload that takes this path in production."""
import ctypes

import numpy as np
import pytest

import minimal_volumetric_path_tracer_amd as vpt
from minimal_volumetric_path_tracer_amd import _lib


def _plan_fn():
    f = vpt.lib().vpt_debug_launch_plan
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.POINTER(_lib.vpt_params), ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_int64]
    return f


def pool_tasks() -> int:
    """task slots per workgroup of this build (vpt_pool.h POOL): 856 with the 11 kill-predicting rings"""
    f = vpt.lib().vpt_debug_pool_tasks
    f.restype = ctypes.c_int
    return int(f())


def clamped(blocks: int, units: int) -> int:
    """launch_pool's workgroup count: no more pools than the units fill"""
    return min(blocks, -(-units // pool_tasks()))


def plan(cfg: vpt.RenderConfig, blocks: int, log2: int = 26):
    f = _plan_fn()
    p = cfg.params()
    n = f(ctypes.byref(p), blocks, log2, None, None, 0)
    assert n >= 1, n
    u0, nu = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    assert f(ctypes.byref(p), blocks, log2, u0.ctypes.data, nu.ctypes.data, n) == n
    return u0.astype(np.int64), nu.astype(np.int64)


def units_of(w, rows, spp):
    """8 x 8-pixel tiles x 64 units each x the auto layout's chunks (csrc/vpt_chunks.h)"""
    C = max(32, (spp + 127) // 128) if spp > 32 else spp
    n, head = 0, spp
    if spp > C:
        head = spp - min(spp, 2 * C)
    n = -(-head // C)
    rem = spp - head
    while rem > 0:
        rem -= (rem + 2) // 3
        n += 1
    return ((w + 7) // 8) * ((rows + 7) // 8) * 64 * n, C


def _check_partition(u0, nu, units):
    assert u0[0] == 0
    assert np.array_equal(u0[1:], u0[:-1] + nu[:-1]), "launches must be contiguous, in unit order"
    assert (nu > 0).all() and u0[-1] + nu[-1] == units
    assert (nu[:-1] == nu[0]).all() and nu[-1] <= nu[0], "every launch but the last is full"


def test_config4_per_gpu_takes_two_launches():
    """configs[4] on 8 GPUs: rank r renders file-row bands r, r + 8, ... (16 rows) = 512 of 4096 rows,
    2^21 pixels; 8192 spp -> 64-sample chunks (126 of them + an 11-chunk taper = 137).  287 M units >
    2^28 = 2^26 samples x 256 workgroups / 64 samples: two launches, the second partial."""
    cfg = vpt.RenderConfig(width=4096, height=4096, spp=8192, estimator="mis", band_rows=16, band_stride=8,
                           band_offset=3)
    assert cfg.shard_rows() == 512
    units, C = units_of(4096, 512, 8192)
    assert C == 64 and units == 2 ** 21 * 137
    u0, nu = plan(cfg, blocks=256)
    _check_partition(u0, nu, units)
    assert len(nu) == 2 and nu[0] == 2 ** 28 and nu[1] == units - 2 ** 28


def test_config1_is_one_launch():
    cfg = vpt.RenderConfig(width=1024, height=1024, spp=256)
    units, _ = units_of(1024, 1024, 256)
    u0, nu = plan(cfg, blocks=256)
    assert len(nu) == 1 and nu[0] == units


@pytest.mark.parametrize("w,h,spp,blocks,log2", [(32, 32, 96, 13, 12), (48, 40, 1024, 7, 10), (8, 6, 5000, 1, 9),
                                                 (17, 9, 33, 3, 5), (64, 64, 256, 256, 0)])
def test_lowered_bound_splits_into_contiguous_launches(w, h, spp, blocks, log2):
    cfg = vpt.RenderConfig(width=w, height=h, spp=spp)
    units, C = units_of(w, h, spp)
    u0, nu = plan(cfg, blocks=blocks, log2=log2)
    _check_partition(u0, nu, units)
    per = max(1, (2 ** log2 * clamped(blocks, units)) // C)
    assert nu[0] == min(per, units) and len(nu) == -(-units // per)


def test_gpu_split_test_geometry_splits():
    """the GPU test's render (tests/test_gpu_parity.py::test_split_launches_equal_one_launch) takes >= 3
    launches for any workgroup count it can get, and at the count launch_pool clamps it to (its units
    over one pool, vpt_debug_pool_tasks) the plan ends in a partial launch"""
    units, C = units_of(32, 32, 96)
    full = -(-units // pool_tasks())
    assert pool_tasks() == 856 and full == 14
    for blocks in range(1, full + 3):
        u0, nu = plan(vpt.RenderConfig(width=32, height=32, spp=96), blocks=blocks, log2=12)
        _check_partition(u0, nu, units)
        assert len(nu) >= 3
        if blocks >= full:  # what launch_pool takes on any GPU with >= 14 CUs: 7 launches, the last partial
            per = (2 ** 12 * full) // C
            assert nu[0] == per and len(nu) == -(-units // per) == 7 and nu[-1] == units - 6 * per < per


def test_bad_arguments_refused():
    f = _plan_fn()
    p = vpt.RenderConfig(width=8, height=8, spp=4).params()
    for blocks, log2 in ((0, 26), (1, -1), (1, 27)):
        assert f(ctypes.byref(p), blocks, log2, None, None, 0) < 0
