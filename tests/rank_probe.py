"""A stand-in rank for tests/test_bench_launch.py: what bench.launch_ranks starts, with the renderer
mocked.  It joins the process group from the environment the launcher set (env://, gloo), "renders"
its row bands as a strip whose every value is its file row index, gathers the strips to rank 0 with
minimal_volumetric_path_tracer_amd.distributed.gather_image (the code bench.py runs), and rank 0 writes
{world, ranks seen, image} to the file named by argv[1].  argv[2] == "fail-rank-1": rank 1 exits 3
before joining (the launcher must fail the run and stop the others)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, mode = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if mode == "fail-rank-1" and rank == 1:
        sys.exit(3)
    if mode == "fail-rank-1":
        time.sleep(60)  # the launcher must stop this rank
    import torch
    import torch.distributed as dist

    from minimal_volumetric_path_tracer_amd import RenderConfig
    from minimal_volumetric_path_tracer_amd.distributed import gather_image, shard_rows

    dist.init_process_group("gloo")
    cfg = RenderConfig(width=4, height=48, spp=1)
    rows = shard_rows(cfg.height, rank, world, 8)
    strip = torch.tensor(rows, dtype=torch.float32)[:, None, None].expand(len(rows), cfg.width, 3).contiguous()
    img = gather_image(strip, cfg, band_rows=8)
    seen = [None] * world
    dist.all_gather_object(seen, {"rank": rank, "world": dist.get_world_size(), "local": os.environ["LOCAL_RANK"],
                                  "master": os.environ["MASTER_ADDR"]})
    if rank == 0:
        json.dump({"world": world, "seen": seen, "image": img[:, 0, 0].tolist()}, open(out, "w"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
