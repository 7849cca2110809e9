"""One rank of tests/test_gpu_multiproc.py, started by bench.launch_ranks: several processes share the
one-GPU box's cuda:0, each renders its row bands through libvpt (gpu_shard_renderer: Tracer on the
device, torch's current stream), copies its strip to host memory, and the strips meet on rank 0 over
gloo through minimal_volumetric_path_tracer_amd.distributed.render_distributed / gather_image -- the
code an N-GPU run executes over RCCL.  Rank 0 saves the image (float32 .npy) to argv[1].

    argv: out.npy estimator width height spp hg_g band_rows"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, est, w, h, spp, g, band = sys.argv[1], sys.argv[2], *map(int, sys.argv[3:6]), float(sys.argv[6]), \
        int(sys.argv[7])
    import numpy as np
    import torch
    import torch.distributed as dist

    import minimal_volumetric_path_tracer_amd as vpt
    from minimal_volumetric_path_tracer_amd.distributed import gpu_shard_renderer, render_distributed

    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t = vpt.Tracer(0)
    try:
        t.set_scene(vpt.default_scene())
        on_gpu = gpu_shard_renderer(t, dev)

        def shard_to_host(scfg):
            strip = on_gpu(scfg)
            return strip.cpu()  # waits for the render on torch's current stream

        cfg = vpt.RenderConfig(width=w, height=h, spp=spp, estimator=est, hg_g=g, seed=0x5EED0001)
        img = render_distributed(cfg, shard_to_host, band_rows=band)
    finally:
        t.close()
    if dist.get_rank() == 0:
        np.save(out, img.numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
