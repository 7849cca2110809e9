"""Henyey-Greenstein phase extension, pinned independently of its restatement.

The reference has only the isotropic phase (include/vptSamplingFunctions.h:34-47 sampler,
include/volumetricBasicFunctions.h:59-62 value 1/(4 pi)); the north-star's HG g (BASELINE.json
configs[2]) is an extension, written twice with the same formula (csrc/vpt_device.h phase_sample /
phase_value, oracle/vpt_oracle.c).  Bitwise GPU == oracle agreement cannot catch a convention error
both share, so these tests check the mathematics itself, on the oracle (CPU) and on the device
(vpt_phase_probe):

  * E[cos theta] = g, cos theta measured against the propagation direction din (4 sigma);
  * a chi-square test of the cos theta histogram against bin probabilities obtained by integrating
    the library's OWN phase_value over each bin -- this ties the sampler to the value the NEE weights
    with (include/volumetricBasicFunctions.h:241,275,300,334 use the phase at mu = din . wl): a
    flipped orientation in either one fails it;
  * the azimuth is uniform around din (the perpendicular component averages to 0);
  * the integral of phase_value over the sphere is 1 (Gauss-Legendre quadrature in mu);
  * g -> 0 tends to the reference's isotropic phase, and g == 0 IS the reference's sampler, bit for bit.
"""
import math

import numpy as np
import pytest

from oracle.oracle import Oracle

GS = (0.9, 0.5, -0.3)
DIN = np.array([0.36, -0.48, 0.8])  # a unit vector away from the axes (din is normalised: 0.36^2 + 0.48^2 + 0.8^2 = 1)


def _states(n, seed=1):
    return np.random.default_rng(seed).integers(0, 2 ** 48, n, dtype=np.uint64)


def _mu_edges(nb=24):
    return np.linspace(-1.0, 1.0, nb + 1)


def _gl(n=512):
    x, w = np.polynomial.legendre.leggauss(n)
    return x, w


def _dirs_at_mu(mu):
    """unit vectors at cosine mu from DIN (azimuth fixed: the value depends on mu only)"""
    d = DIN / np.linalg.norm(DIN)
    a = np.array([1.0, 0.0, 0.0])
    t = np.cross(d, a)
    t /= np.linalg.norm(t)
    s = np.sqrt(np.maximum(0.0, 1.0 - mu * mu))
    return mu[:, None] * d[None, :] + s[:, None] * t[None, :]


def _bin_probs(value_fn, g, edges):
    """P(mu in bin) = 2 pi * integral of the library's phase_value over the bin (GL per bin)"""
    x, w = _gl(64)
    probs = []
    for a, b in zip(edges[:-1], edges[1:]):
        mu = 0.5 * (b - a) * x + 0.5 * (b + a)
        v = value_fn(g, _dirs_at_mu(mu))
        probs.append(2 * math.pi * 0.5 * (b - a) * float((w * v).sum()))
    return np.array(probs)


def _check_distribution(dirs, value_fn, g):
    d = DIN / np.linalg.norm(DIN)
    mu = dirs @ d
    n = len(mu)
    assert np.allclose(np.linalg.norm(dirs, axis=1), 1.0, atol=1e-12)
    # E[cos theta] = g (HG's defining moment), 4 sigma
    m, sd = mu.mean(), mu.std()
    assert abs(m - g) < 4 * sd / math.sqrt(n) + 1e-12, (g, m)
    # chi-square against the library's own value, integrated per bin
    edges = _mu_edges()
    p = _bin_probs(value_fn, g, edges)
    assert abs(p.sum() - 1.0) < 1e-6
    obs, _ = np.histogram(mu, bins=edges)
    exp = p * n
    chi2 = float(((obs - exp) ** 2 / exp).sum())
    assert chi2 < 70.0, (g, chi2)  # 23 dof: P(chi2 > 70) ~ 1e-6
    # uniform azimuth: the component of the direction perpendicular to din averages to 0
    perp = dirs - mu[:, None] * d[None, :]
    assert np.all(np.abs(perp.mean(0)) < 4 * perp.std(0) / math.sqrt(n) + 1e-12)


def _check_normalisation(value_fn, g):
    x, w = _gl(2048)
    v = value_fn(g, _dirs_at_mu(x))
    total = 2 * math.pi * float((w * v).sum())
    assert abs(total - 1.0) < 1e-7, (g, total)


# ------------------------------------------------------------------ oracle (CPU)
@pytest.fixture(scope="module")
def orc():
    return Oracle(portable=True)


def _orc_value(orc):
    return lambda g, wl: orc.hg_phase(g, DIN, np.zeros(0, dtype=np.uint64), wl)[2]


@pytest.mark.parametrize("g", GS)
def test_oracle_hg_distribution(orc, g):
    dirs, _, _ = orc.hg_phase(g, DIN, _states(60000, seed=int(1000 * abs(g)) + 7), np.zeros((0, 3)))
    _check_distribution(dirs, _orc_value(orc), g)


@pytest.mark.parametrize("g", GS + (1e-7,))
def test_oracle_hg_normalisation(orc, g):
    _check_normalisation(_orc_value(orc), g)


def test_oracle_hg_small_g_tends_to_isotropic(orc):
    wl = _dirs_at_mu(np.linspace(-1, 1, 33))
    v = orc.hg_phase(1e-9, DIN, np.zeros(0, dtype=np.uint64), wl)[2]
    assert np.allclose(v, 1 / (4 * math.pi), rtol=1e-8)
    dirs, _, _ = orc.hg_phase(1e-9, DIN, _states(40000, seed=3), np.zeros((0, 3)))
    mu = dirs @ (DIN / np.linalg.norm(DIN))
    obs, _ = np.histogram(mu, bins=_mu_edges())
    exp = len(mu) / len(obs)
    assert float(((obs - exp) ** 2 / exp).sum()) < 70.0
    assert abs(mu.mean()) < 4 * mu.std() / math.sqrt(len(mu))


def test_oracle_g0_is_the_reference_sampler(orc):
    """g == 0: the reference's isotropicPhaseSample (world frame, draws xi1, xi2) and 1/(4 pi)."""
    st = _states(257, seed=5)
    dirs, end, vals = orc.hg_phase(0.0, DIN, st, _dirs_at_mu(np.array([-0.5, 0.0, 0.7])))
    iso = np.zeros(3)
    for i, s in enumerate(st):
        e = orc.L.orc_isotropic_phase(int(s), iso.ctypes.data)
        assert np.array_equal(dirs[i], iso) and int(end[i]) == e
    assert np.all(vals == 1 / (4 * math.pi))
    try:
        from oracle.oracle import Reference
        ref = Reference()
    except (FileNotFoundError, OSError):
        pytest.skip("oracle/_ref not built")
    for i, s in enumerate(st[:64]):
        e = ref.L.ref_isotropic_phase(int(s), iso.ctypes.data)
        assert np.array_equal(dirs[i], iso) and int(end[i]) == e


# ------------------------------------------------------------------ device
@pytest.fixture(scope="module")
def tracer():
    import minimal_volumetric_path_tracer_amd as vpt
    t = vpt.Tracer(0)
    yield t
    t.close()


def _gpu_value(tracer):
    return lambda g, wl: tracer.hg_phase(g, DIN, np.zeros(0, dtype=np.uint64), wl)[2]


@pytest.mark.gpu
@pytest.mark.parametrize("g", GS)
def test_gpu_hg_distribution(tracer, g):
    dirs, _, _ = tracer.hg_phase(g, DIN, _states(1 << 20, seed=int(1000 * abs(g)) + 11), np.zeros((0, 3)))
    _check_distribution(dirs, _gpu_value(tracer), g)


@pytest.mark.gpu
@pytest.mark.parametrize("g", GS + (1e-7,))
def test_gpu_hg_normalisation(tracer, g):
    _check_normalisation(_gpu_value(tracer), g)


@pytest.mark.gpu
@pytest.mark.parametrize("g", (0.0,) + GS)
def test_gpu_hg_bitwise_vs_oracle(tracer, orc, g):
    st = _states(4096, seed=9)
    wl = _dirs_at_mu(np.linspace(-1, 1, 129))
    d0, e0, v0 = tracer.hg_phase(g, DIN, st, wl)
    d1, e1, v1 = orc.hg_phase(g, DIN, st, wl)
    assert np.array_equal(d0, d1) and np.array_equal(e0, e1) and np.array_equal(v0, v1)
