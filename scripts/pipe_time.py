"""Step time of back-to-back renders of the 1/N row-band shard (as bench.py --gpus N), serialized on
one stream vs `depth` contexts on their own streams (a launch's drain overlapped with the next
launch's start).  usage: python scripts/pipe_time.py [config] [N...]"""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import minimal_volumetric_path_tracer_amd as vpt
from bench import CONFIGS

cname = sys.argv[1] if len(sys.argv) > 1 else "ff"
Ns = [int(a) for a in sys.argv[2:]] or [1, 8]
c = CONFIGS[cname]
K = int(os.environ.get("STEPS", "12"))
DEPTHS = [int(x) for x in os.environ.get("DEPTHS", "1,2,3").split(",")]
trs = [vpt.Tracer(0) for _ in range(max(DEPTHS))]
streams = [torch.cuda.Stream() for _ in range(max(DEPTHS))]
for N in Ns:
    cfg = vpt.RenderConfig(**c, seed=0x5EED0001, band_rows=16 if N > 1 else c["height"], band_stride=N, band_offset=0)
    outs = [torch.empty((cfg.shard_rows(), c["width"], 3), dtype=torch.float32, device="cuda") for _ in range(max(DEPTHS))]
    res = {}
    for depth in DEPTHS:
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                j = k % depth
                trs[j].render_device(cfg, outs[j].data_ptr(), streams[j].cuda_stream)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / K * 1e3
        res[depth] = dt
        same = all(torch.equal(outs[0], outs[j]) for j in range(depth))
        print(f"{cname} 1/{N} depth {depth}: {dt:.3f} ms/step  (images identical: {same})", flush=True)
