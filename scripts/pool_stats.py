"""Debug: scheduler statistics of the pool kernel (VPT_POOL_STATS=1, layout in csrc/vpt_pool.h)."""
import ctypes, os, sys, time
os.environ["VPT_POOL_STATS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VPT_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build_variants", "libvpt_dbg.so"))
import minimal_volumetric_path_tracer_amd as vpt

NSTATS = 24
RINGS = ["A", "S dif/sph", "S dif/pt", "S metal", "S other", "M sph", "M pt"]
t = vpt.Tracer(0)
est = sys.argv[1] if len(sys.argv) > 1 else "ff"
g = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
sizes = [(1024, 1024, 256 if est == "ff" else 128)]
for w, h, spp in sizes:
    t.render(width=64, height=64, spp=4, estimator=est, hg_g=g)
    buf0 = (ctypes.c_ulonglong * NSTATS)()
    vpt.lib().vpt_debug_pool_stats(buf0)  # (reads and clears, if the build clears)
    t0 = time.time()
    t.render(width=w, height=h, spp=spp, estimator=est, hg_g=g)
    dt = time.time() - t0
    buf = (ctypes.c_ulonglong * NSTATS)()
    vpt.lib().vpt_debug_pool_stats(buf)
    s = list(buf)
    b, l, cyc = s[0:7], s[7:14], s[16:20]
    tot = max(sum(cyc), 1)
    nA = max(b[0], 1)
    print(f"{w}x{h}x{spp}: {dt*1e3:.1f} ms {w*h*spp/dt/1e6:.1f} Ms/s (instrumented)")
    for r in range(7):
        print(f"  ring {RINGS[r]:10s} batches {b[r]:9d} mean lanes {l[r]/max(b[r],1):5.1f}")
    print(f"  cycle share A/S/M/sched {[round(c/tot, 3) for c in cyc]}  idle polls {s[14]} ticket waits {s[15]}")
    sb, mb = max(sum(b[1:5]), 1), max(sum(b[5:7]), 1)
    print(f"  cycles per batch A {cyc[0]/nA:.0f} S {cyc[1]/sb:.0f} M {cyc[2]/mb:.0f}")
    print(f"  stage A: prep rounds/batch {s[20]/nA:.2f} prep cycles/batch {s[22]/nA:.0f}"
          f" decide cycles/batch {s[23]/nA:.0f} samples {s[21]} (expect {w*h*spp})", flush=True)
