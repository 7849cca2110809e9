"""Debug: section-timer shares of the pool kernel (a build with -DVPT_SECTIONS=1, csrc/vpt_device.h).
usage: VPT_LIB=build_variants/libvpt_sect.so python scripts/sect_stats.py [ff|mis] [hg_g]"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import minimal_volumetric_path_tracer_amd as vpt

NAMES = ["sched", "load_task", "S pLight", "S MISv2", "S MISv2 isect3", "S bdsf+update", "M single_scat", "M ss cone dir",
         "M ss cone isect", "M ss shadow/Ld", "M phase", "roulette", "A prep", "A decide", "A decide isect", "store_task",
         "S total", "M total", "A camera", "A decide (in)", "M shadow (in)", "A camera (in)", "M eqa",
         "M transmittance", "A unit handout", "A rounds >= 2"]
N = 32
t = vpt.Tracer(0)
est = sys.argv[1] if len(sys.argv) > 1 else "ff"
g = float(sys.argv[2]) if len(sys.argv) > 2 else (0.5 if est == "mis" else 0.0)
spp = 256 if est == "ff" else 128
t.render(width=64, height=64, spp=4, estimator=est, hg_g=g)
buf = (ctypes.c_ulonglong * (3 * N))()
vpt.lib().vpt_debug_sections(buf)
t0 = time.time()
t.render(width=1024, height=1024, spp=spp, estimator=est, hg_g=g)
dt = time.time() - t0
vpt.lib().vpt_debug_sections(buf)
s = list(buf)
top = max(1, s[0] + s[1] + s[16] + s[17] + s[11] + s[12] + s[18] + s[13] + s[15])
print(f"{est} g={g} 1024x1024x{spp}: {dt*1e3:.1f} ms (instrumented); top-level wave-cycles {top:.3e}")
for k, name in enumerate(NAMES):
    c, n = s[k], s[N + k]
    if n:
        print(f"  {name:16s} share {c/top:6.3f}  entries {n:10d}  cycles/entry {c/n:8.0f}  lanes/entry {s[2 * N + k]/n:5.1f}")
