"""TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg): times the reference's own estimator
(oracle/_ref/libvpt_ref.so, ref_harness.cpp) on some file rows of an image, in this process, and
prints the render time in seconds.

bench.py starts one such process per core.  The harness drives the reference's global erand48
state (include/Vector.h:38), so the parallel measurement uses one process per core, not threads.

usage: python -m oracle.ref_rate EST W H SPP SIGMA_A SIGMA_S ROW [ROW ...]   (ROW: file rows)
"""
import sys
import time

from oracle.oracle import Reference


def main() -> None:
    est, w, h, spp = (int(a) for a in sys.argv[1:5])
    sa, ss = float(sys.argv[5]), float(sys.argv[6])
    rows = [int(r) for r in sys.argv[7:]]
    ref = Reference()
    ref.set_scene(ref.default_scene())
    t = time.perf_counter()
    for fr in rows:
        y = h - 1 - fr  # camera row of file row fr (src/rt.cpp:773)
        ref.render(w, h, spp, est, sa, ss, seed=0x5EED0001, y0=y, y1=y + 1)
    print(f"{time.perf_counter() - t:.6f}")


if __name__ == "__main__":
    main()
