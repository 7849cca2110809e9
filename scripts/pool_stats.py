"""Debug: scheduler statistics of the pool kernel (VPT_POOL_STATS=1, layout in csrc/vpt_pool.h)."""
import ctypes, os, sys, time
os.environ["VPT_POOL_STATS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import minimal_volumetric_path_tracer_amd as vpt

NSTATS = 24
t = vpt.Tracer(0)
sizes = [(256, 256, 64), (1024, 1024, 64), (1024, 1024, 256)]
for w, h, spp in sizes:
    t0 = time.time()
    t.render(width=w, height=h, spp=spp)
    dt = time.time() - t0
    s = list((ctypes.c_ulonglong * NSTATS)())
    buf = (ctypes.c_ulonglong * NSTATS)()
    vpt.lib().vpt_debug_pool_stats(buf)
    s = list(buf)
    b, l, cyc = s[0:3], s[3:6], s[8:12]
    tot = sum(cyc)
    print(f"{w}x{h}x{spp}: {dt*1e3:.1f} ms {w*h*spp/dt/1e6:.1f} Ms/s")
    print(f"  batches A/S/M {b} mean lanes {[round(l[i]/max(b[i],1),1) for i in range(3)]}"
          f" idle polls {s[6]} ticket waits {s[7]}")
    print(f"  cycle share A/S/M/sched {[round(c/max(tot,1),3) for c in cyc]}"
          f"  cycles per batch A/S/M {[round(cyc[i]/max(b[i],1)) for i in range(3)]}")
    print(f"  stage A: prep rounds/batch {s[12]/max(b[0],1):.2f} decide lanes/batch {s[14]/max(b[0],1):.1f}"
          f" samples {s[15]} (expect {w*h*spp})")
    print(f"  stage A cycles/batch: prep {s[16]/max(b[0],1):.0f} decide {s[18]/max(b[0],1):.0f}"
          f" load+store {s[19]/max(b[0],1):.0f}")
    r = max(s[12], 1)
    print(f"  prep round: grab section {s[17]/r:.0f} cycles, sample-start section {s[20]/r:.0f} cycles,"
          f" rounds with a queue atomic {s[21]/r:.3f}", flush=True)
