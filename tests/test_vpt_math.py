"""The path's libm as the oracle's portable build evaluates it (lm_* of csrc/vpt_math.h: the
glibc-exact restatement of csrc/vpt_glibm.h, the same source the kernel compiles) against the
host's glibc: within 3 ulp everywhere on the tracer's ranges (tests/test_glibc_libm.py holds the
bit-exact bar), special values handled like C99 Annex F."""
import numpy as np
import pytest


def ulps(a, b):
    a, b = np.asarray(a), np.asarray(b)
    both_nan = np.isnan(a) & np.isnan(b)
    same = (a == b) | both_nan
    sp = np.spacing(np.maximum(np.abs(b), np.finfo(float).tiny))
    d = np.where(same, 0.0, np.abs(a - b) / sp)
    return np.where(np.isnan(d), np.inf, d)


CASES = [
    (1, "exp", [(-745, 710), (-50, 0), (-1, 1)]),
    (2, "log", [(1e-300, 1e-200), (1e-12, 1.0), (0.5, 2.0), (1.0, 1e300)]),
    (3, "sin", [(0, 2 * np.pi), (-100, 100)]),
    (4, "cos", [(0, 2 * np.pi), (-100, 100)]),
    (5, "tan", [(-1.5, 1.5)]),
    (6, "atan", [(-1, 1), (-60, 60), (0, 1e12)]),
    (7, "acos", [(-1, 1), (0.999, 1.0), (-1.0, -0.999)]),
]


@pytest.mark.parametrize("fn,name,ranges", CASES)
def test_within_3_ulp_of_glibc(orc, orc_vm, fn, name, ranges):
    rng = np.random.default_rng(fn)
    for lo, hi in ranges:
        x = rng.uniform(lo, hi, 100000)
        u = ulps(orc_vm.math(fn, x), orc.math(fn, x))
        assert u.max() <= 3, f"{name} on [{lo},{hi}]: {u.max()} ulp"
        assert (u == 0).mean() > 0.55, f"{name}: only {(u == 0).mean():.2f} identical to glibc"


def test_atan2_quadrants(orc, orc_vm):
    rng = np.random.default_rng(8)
    y = rng.uniform(-100, 100, 100000)
    x = rng.uniform(-100, 100, 100000)
    assert ulps(orc_vm.math(8, y, x), orc.math(8, y, x)).max() <= 3
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan])
    Y, X = np.meshgrid(sp, sp)
    a, b = orc_vm.math(8, Y.ravel(), X.ravel()), orc.math(8, Y.ravel(), X.ravel())
    assert (ulps(a, b) <= 1).all()
    assert np.array_equal(np.signbit(a[~np.isnan(a)]), np.signbit(b[~np.isnan(b)]))


def test_special_values(orc, orc_vm):
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-310, -1e-310, 710.0, -746.0, 2.0])
    for fn in (1, 2, 3, 4, 5, 6, 7):
        a, b = orc_vm.math(fn, sp), orc.math(fn, sp)
        assert (ulps(a, b) <= 1).all(), (fn, a, b)
    # the values the tracer depends on exactly
    assert orc_vm.math(7, np.array([1.0]))[0] == 0.0          # acos(1): point-light cone
    assert orc_vm.math(2, np.array([1.0]))[0] == 0.0          # log(1): xi = 0 free flight
    assert orc_vm.math(1, np.array([0.0]))[0] == 1.0
    s = orc_vm.math(3, np.array([0.0]))[0]
    assert s == 0.0 and orc_vm.math(4, np.array([0.0]))[0] == 1.0
