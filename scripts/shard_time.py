"""Per-rank kernel time of the N-GPU strong-scaling split, measured on one GPU: rank r of N renders
file-row bands r, r+N, ... (16 rows each), exactly as bench.py --gpus N does; compares N x that
time with the whole image (ideal: equal).  usage: python scripts/shard_time.py [config] [N...]"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import minimal_volumetric_path_tracer_amd as vpt
from bench import CONFIGS

cname = sys.argv[1] if len(sys.argv) > 1 else "ff"
Ns = [int(a) for a in sys.argv[2:]] or [1, 2, 4, 8]
c = CONFIGS[cname]
tr = vpt.Tracer(0)
stream = torch.cuda.current_stream()


def timed(cfg, reps=3):
    out = torch.empty((cfg.shard_rows(), c["width"], 3), dtype=torch.float32, device="cuda")
    tr.render_device(cfg, out.data_ptr(), stream.cuda_stream)
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        tr.render_device(cfg, out.data_ptr(), stream.cuda_stream)
        b.record(stream)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    return min(ms)


BAND = int(os.environ.get("BAND_ROWS", "16"))
base = None
for N in Ns:
    worst = 0.0
    per = []
    for r in (range(N) if os.environ.get("ALL_RANKS") else ([0, N - 1] if N > 1 else [0])):
        cfg = vpt.RenderConfig(**c, seed=0x5EED0001, chunk_spp=int(os.environ.get("CHUNK", "0")), band_rows=BAND if N > 1 else c["height"], band_stride=N, band_offset=r)
        per.append(timed(cfg))
    worst = max(per)
    if len(per) > 2:
        print("  per rank ms:", " ".join(f"{x:.3f}" for x in per))
    if base is None:
        base = worst * N
    print(f"{cname} chunk {os.environ.get('CHUNK', '0')} band {BAND} N={N}: slowest probed rank {worst:.3f} ms  -> ideal-scaling efficiency {base / (N * worst):.3f}", flush=True)
