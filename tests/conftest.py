import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(TESTS, "golden")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvpt.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _ensure_built():
    need = [
        os.path.join(ROOT, "oracle", "liboracle.so"),
        os.path.join(ROOT, "oracle", "liboracle_vm.so"),
        os.path.join(ROOT, "minimal_volumetric_path_tracer_amd", "libvpt.so"),
    ]
    if not all(os.path.exists(p) for p in need):
        import __graft_entry__

        __graft_entry__.build()


_ensure_built()


@pytest.fixture(scope="session")
def samples():
    return dict(np.load(os.path.join(GOLDEN, "samples.npz")))


@pytest.fixture(scope="session")
def samples_e234():
    """per-sample KATs + framebuffers of estimators 2-4 (tests/golden/make_golden.py --estimators-234)"""
    return dict(np.load(os.path.join(GOLDEN, "samples_e234.npz")))


@pytest.fixture(scope="session")
def samples_alt():
    """the reference's alternate scenes x all five estimators (make_golden.py --alt-scenes)"""
    return dict(np.load(os.path.join(GOLDEN, "samples_alt.npz")))


@pytest.fixture(scope="session")
def samples_e5():
    """iterativePathTracer (estimator 5) on the test + alternate scenes (make_golden.py --surface-pt)"""
    return dict(np.load(os.path.join(GOLDEN, "samples_e5.npz")))


@pytest.fixture(scope="session")
def samples_e6():
    """rayMarching3 (estimator 6) cases of make_golden.py MARCH_CASES (make_golden.py --ray-marching)"""
    return dict(np.load(os.path.join(GOLDEN, "samples_e6.npz")))


@pytest.fixture(scope="session")
def samples_e789():
    """rayMarching2 / rayMarchingGlobal / rayMarching (estimators 7-9), punctualVolumetric and
    rayMarching's out-parameters (make_golden.py --ray-marching-789)"""
    return dict(np.load(os.path.join(GOLDEN, "samples_e789.npz")))


@pytest.fixture(scope="session")
def prims():
    return dict(np.load(os.path.join(GOLDEN, "primitives.npz")))


@pytest.fixture(scope="session", params=["libm", "portable"])
def orc(request):
    """both oracle builds: libm (glibc calls) and portable (csrc/vpt_math.h lm_*, the HIP kernel's
    arithmetic: glibc's algorithms restated).  The two are the same function bit for bit, so every
    reference bar holds for the arithmetic the GPU executes."""
    from oracle.oracle import Oracle

    return Oracle(portable=request.param == "portable")


@pytest.fixture(scope="session")
def orc_vm():
    from oracle.oracle import Oracle

    return Oracle(portable=True)


@pytest.fixture(scope="session")
def gpu_tracer():
    from minimal_volumetric_path_tracer_amd import Tracer

    t = Tracer(0)
    yield t
    t.close()


def bitwise_equal(a, b):
    """elementwise identical bits, NaN == NaN (any payload), -0.0 == +0.0 only when both zero"""
    a = np.asarray(a)
    b = np.asarray(b)
    return (a == b) | (np.isnan(a) & np.isnan(b))
