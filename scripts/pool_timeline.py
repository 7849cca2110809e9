"""Debug: per-workgroup timeline of one pool_kernel launch (VPT_POOL_DEBUG=2 build, VPT_POOL_STATS=1):
when each workgroup started, first saw the global work queue exhausted, and exited (vpt_pool.h TL0).
usage: python scripts/pool_timeline.py [config] [N]   (N: render the 1/N row-band shard of bench.py --gpus N)"""
import ctypes, os, sys
os.environ["VPT_POOL_STATS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("VPT_LIB", os.path.join(ROOT, "build_variants", "libvpt_dbg2.so"))
import numpy as np
import minimal_volumetric_path_tracer_amd as vpt
from bench import CONFIGS

cname = sys.argv[1] if len(sys.argv) > 1 else "ff"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1
c = CONFIGS[cname]
t = vpt.Tracer(0)
cfg = vpt.RenderConfig(**c, seed=0x5EED0001, band_rows=16 if N > 1 else c["height"], band_stride=N, band_offset=0)
for rep in range(2):
    t.render(cfg)
buf = (ctypes.c_ulonglong * (3 * 4096))()
vpt.lib().vpt_debug_pool_timeline(buf)
a = np.array(buf, dtype=np.uint64).reshape(4096, 3)
used = a[:, 0] != np.uint64(0xFFFFFFFFFFFFFFFF)
a = a[used]
start = a[:, 0].astype(np.float64)
exh = np.where(a[:, 1] == np.uint64(0xFFFFFFFFFFFFFFFF), np.nan, a[:, 1].astype(np.float64))
end = (~a[:, 2]).astype(np.float64)
t0 = start.min()
us = lambda x: (x - t0) / 100.0  # 100 MHz -> us
print(f"{cname} 1/{N}: {used.sum()} workgroups")
for name, x in (("start", us(start)), ("queue exhausted", us(exh)), ("exit", us(end))):
    q = np.nanpercentile(x, [0, 10, 50, 90, 100])
    print(f"  {name:16s} us  min {q[0]:9.1f}  p10 {q[1]:9.1f}  p50 {q[2]:9.1f}  p90 {q[3]:9.1f}  max {q[4]:9.1f}")
print(f"  drain (exit - first exhaustion) per WG: p50 {np.nanmedian(us(end) - us(exh)):.1f} us; "
      f"kernel span {us(end).max():.1f} us; last exhaustion -> last exit {us(end).max() - np.nanmax(us(exh)):.1f} us")
