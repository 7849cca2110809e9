"""vpt_multi_render's reassembly of gathered strips into file order (vpt_debug_band_reorder, the
code the n > 1 path runs after the RCCL gather), on the CPU: for any device count and band size the
strips cut by the band layout (vpt_shard_rows) go back to the image byte for byte."""
import ctypes

import numpy as np
import pytest

import minimal_volumetric_path_tracer_amd as vpt


def _reorder():
    L = vpt.lib()
    f = L.vpt_debug_band_reorder
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                  ctypes.c_void_p]
    return f


def _shard_rows(h, band, n, g):
    return [fr for fr in range(h) if (fr // band) % n == g]


@pytest.mark.parametrize("n,band,h", [(1, 768, 768), (2, 16, 768), (3, 16, 70), (8, 16, 1024), (8, 5, 53),
                                      (7, 1, 29), (8, 16, 9)])
def test_band_reorder_restores_file_order(n, band, h):
    w = 5
    img = np.random.default_rng(n * 100 + band).random((h, w, 3)).astype(np.float32)
    rows = [_shard_rows(h, band, n, g) for g in range(n)]
    for g in range(n):  # the library's own shard size for the same layout
        p = vpt.RenderConfig(width=w, height=h, band_rows=band, band_stride=n, band_offset=g).params()
        assert vpt.lib().vpt_shard_rows(ctypes.byref(p)) == len(rows[g])
    cap = max(1, max(len(r) for r in rows))
    staging = np.zeros((n, cap, w, 3), dtype=np.float32)
    for g in range(n):
        staging[g, :len(rows[g])] = img[rows[g]]
    out = np.zeros_like(img)
    row_bytes = w * 3 * 4
    assert _reorder()(staging.ctypes.data, cap * row_bytes, n, h, band, row_bytes, out.ctypes.data) == 0
    assert out.tobytes() == img.tobytes()


def test_band_reorder_rejects_short_slots():
    st = np.zeros(10, dtype=np.float32)
    out = np.zeros(40, dtype=np.float32)
    assert _reorder()(st.ctypes.data, 8, 2, 10, 1, 4, out.ctypes.data) != 0  # slot holds 2 rows, needs 5
