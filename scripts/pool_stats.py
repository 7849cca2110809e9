"""Debug: scheduler statistics of the pool kernel (VPT_POOL_STATS=1)."""
import ctypes, os, sys, time
os.environ["VPT_POOL_STATS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import minimal_volumetric_path_tracer_amd as vpt

t = vpt.Tracer(0)
for w, h, spp in [(128, 128, 16), (256, 256, 64)]:
    t0 = time.time()
    img = t.render(width=w, height=h, spp=spp)
    dt = time.time() - t0
    s = (ctypes.c_ulonglong * 8)()
    vpt.lib().vpt_debug_pool_stats(s)
    b, l = list(s[0:3]), list(s[3:6])
    print(f"{w}x{h}x{spp}: {dt*1e3:.1f} ms  {w*h*spp/dt/1e6:.1f} Ms/s  batches A/S/M {b}  mean lanes "
          f"{[round(l[i]/max(b[i],1),1) for i in range(3)]}  idle polls {s[6]}  lock retries {s[7]}", flush=True)
