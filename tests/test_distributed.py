"""N > 1 path on CPU: two (and three) gloo ranks render their row bands and gather the image to
rank 0 through minimal_volumetric_path_tracer_amd.distributed -- the same code bench.py and
multi-GPU users run over RCCL.  The per-rank renderer here is the oracle (test infrastructure);
on the GPU it is libvpt.  The gathered image must equal the single-process render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from minimal_volumetric_path_tracer_amd import RenderConfig
from minimal_volumetric_path_tracer_amd.distributed import assemble, render_distributed, shard_config, shard_rows

W, H, SPP, SEED = 24, 40, 2, 17


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_shard(scfg: RenderConfig) -> torch.Tensor:
    from oracle.oracle import Oracle
    from scenes import SCENES

    o = Oracle(portable=True)
    o.set_scene(SCENES["default"]())
    full = o.render(scfg.width, scfg.height, scfg.spp, 0, seed=scfg.seed, threads=1)
    rows = shard_rows(scfg.height, scfg.band_offset, scfg.band_stride, scfg.band_rows) if scfg.band_stride > 1 \
        else list(range(scfg.height))
    return torch.from_numpy(full[rows].astype(np.float32))


def _worker(rank, world, port, band, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    cfg = RenderConfig(width=W, height=H, spp=SPP, seed=SEED)
    img = render_distributed(cfg, _oracle_shard, band_rows=band)
    if rank == 0:
        q.put(img.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 8), (2, 16), (3, 4)])
def test_gloo_gather_equals_single_process(world, band):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _oracle_shard(RenderConfig(width=W, height=H, spp=SPP, seed=SEED)).numpy()
    assert img.shape == (H, W, 3)
    assert np.array_equal(img, ref)


def test_assemble_and_shard_configs():
    full = torch.arange(H * W * 3, dtype=torch.float32).reshape(H, W, 3)
    for world, band in [(2, 8), (4, 16), (5, 3), (8, 16)]:
        parts = [full[shard_rows(H, r, world, band)] for r in range(world)]
        assert torch.equal(assemble(parts, H, band), full)
        cfg = RenderConfig(width=W, height=H)
        assert sum(shard_config(cfg, r, world, band).shard_rows() for r in range(world)) == H


def test_assemble_builds_its_row_indices_once(monkeypatch):
    """the per-image reassembly on rank 0 reuses its row-index tensors (built on the first image of a
    layout): building them per image is a blocking host-to-device copy on a GPU rank"""
    import minimal_volumetric_path_tracer_amd.distributed as d

    full = torch.arange(H * W * 3, dtype=torch.float32).reshape(H, W, 3)
    world, band = 4, 8
    parts = [full[shard_rows(H, r, world, band)] for r in range(world)]
    monkeypatch.setattr(d, "_ROW_INDEX", {})
    assert torch.equal(assemble(parts, H, band), full)
    built = dict(d._ROW_INDEX)
    calls = []
    real = torch.tensor
    monkeypatch.setattr(torch, "tensor", lambda *a, **k: calls.append(1) or real(*a, **k))
    assert torch.equal(assemble(parts, H, band), full)
    assert calls == [] and d._ROW_INDEX.keys() == built.keys()
