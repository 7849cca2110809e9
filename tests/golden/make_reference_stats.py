#!/usr/bin/env python3
"""Statistical fixtures of the REFERENCE PROGRAM itself (SURVEY 8c fixture 4, 8d iii).

The reference's own output is a Monte Carlo image from an entropy-seeded RNG (src/rt.cpp:746,
include/Vector.h:38): no two runs agree, so the product is pinned to it statistically.
  1. `oracle/_ref/rt_tls 16` -- src/rt.cpp unchanged (1024x768, 16 spp, free flight, image.ppm)
     except that the erand48 state is per thread (BASELINE.md's per-thread-RNG flavour, see
     below) -- is run RUNS times; stored: the 8-bit image of run 0, every run's per-channel 8-bit
     mean, and the run-to-run per-channel RMSE of the 8-bit images (all pairs).
     The program as written (`oracle/_ref/rt`, one erand48 state shared by all OpenMP threads
     without synchronisation) is run RACY_RUNS times for its 8-bit means only: the data
     race duplicates and skips draws, and its image is measurably brighter (red +0.25, blue +0.2
     of 255, ~5 sigma of a 16-spp image), so it is recorded, not used as the pin.
  Both programs are built with -ffp-contract=off (oracle/Makefile).
  2. The reference's own estimators through the harness (oracle/_ref/libvpt_ref.so) at 64x64 and
     high spp, free flight and MIS: per-channel linear image mean and its standard error (from the
     per-sample values: mean over pixels of the within-pixel sample variance / samples).
Only program outputs and statistics are stored (no reference source).

    python tests/golden/make_reference_stats.py      # writes tests/golden/reference_stats.npz
"""
from __future__ import annotations

import itertools
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.oracle import Reference  # noqa: E402

RUNS = 4
RACY_RUNS = 2
PROG_SPP = 16
HARNESS = dict(w=64, h=64, spp=1024, seed=0x5EED00AA)


def read_ppm(path: str) -> np.ndarray:
    data = open(path, "rb").read().split()
    assert data[0] == b"P3"
    w, h = int(data[1]), int(data[2])
    vals = np.array(data[4:], dtype=np.int64)
    assert len(vals) == w * h * 3
    return vals.reshape(h, w, 3).astype(np.uint8)


def program_runs(name: str, runs: int) -> list[np.ndarray]:
    exe = os.path.join(ROOT, "oracle", "_ref", name)
    imgs = []
    env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
    for k in range(runs):
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([exe, str(PROG_SPP)], cwd=d, capture_output=True, text=True, env=env, check=True)
            assert r.stdout.startswith("elapsed time: "), r.stdout
            imgs.append(read_ppm(os.path.join(d, "image.ppm")))
        print(f"{name} run {k}: {r.stdout.strip()}", flush=True)
    return imgs


def harness_stats(ref: Reference, est: int) -> tuple[np.ndarray, np.ndarray]:
    w, h, spp = HARNESS["w"], HARNESS["h"], HARNESS["spp"]
    img, ps = ref.render(w, h, spp, est, seed=HARNESS["seed"], per_sample=True)
    ps = ps.reshape(h * w, spp, 3)
    mean = img.reshape(-1, 3).mean(0)
    se = np.sqrt(ps.var(axis=1, ddof=1).mean(0) / (h * w * spp))
    return mean, se


def main() -> None:
    imgs = program_runs("rt_tls", RUNS)
    means = np.array([im.reshape(-1, 3).mean(0) for im in imgs])
    racy_means = np.array([im.reshape(-1, 3).mean(0) for im in program_runs("rt", RACY_RUNS)])
    pair_rmse = np.array([np.sqrt(((a.astype(np.float64) - b) ** 2).reshape(-1, 3).mean(0))
                          for a, b in itertools.combinations(imgs, 2)])
    ref = Reference()
    ref.set_scene(ref.default_scene())
    m0, s0 = harness_stats(ref, 0)
    m1, s1 = harness_stats(ref, 1)
    out = os.path.join(HERE, "reference_stats.npz")
    np.savez_compressed(out, run0=imgs[0], run_means=means, pair_rmse=pair_rmse, prog_spp=PROG_SPP,
                        racy_run_means=racy_means,
                        harness_wh_spp=np.array([HARNESS["w"], HARNESS["h"], HARNESS["spp"]]),
                        harness_seed=np.uint64(HARNESS["seed"]), ff_mean=m0, ff_se=s0, mis_mean=m1, mis_se=s1)
    print("racy program 8-bit means", racy_means)
    print("8-bit run means", means, "\nrun-to-run rmse", pair_rmse.mean(0), "max", pair_rmse.max(0))
    print("harness ff", m0, s0, "mis", m1, s1)
    print("wrote", out)


if __name__ == "__main__":
    main()
