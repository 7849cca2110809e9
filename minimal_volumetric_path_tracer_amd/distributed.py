"""Multi-GPU rendering: one process per GPU, image rows sharded, strips gathered to rank 0.

Every (pixel, sample) owns its random stream (csrc/vpt_rng.h) and every pixel is accumulated by
exactly one lane in sample order, so the image is bit-identical for any number of GPUs and any
band layout (tests/test_gpu_parity.py::test_shards_compose_bitwise, tests/test_distributed.py).
The only exchange is one gather of float32 strips to rank 0 over RCCL (torch.distributed
"nccl"); there is no data-path collective.

Layout: file rows (row 0 = top, src/rt.cpp:773) are cut into bands of `band_rows`; rank r
renders bands r, r+world, r+2*world, ... (interleaving balances the per-band cost, which varies
by ~8 % across the reference image) into one compact strip.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, Optional

import torch

from .tracer import RenderConfig

DEFAULT_BAND_ROWS = 16


def shard_config(cfg: RenderConfig, rank: int, world: int, band_rows: int = DEFAULT_BAND_ROWS) -> RenderConfig:
    """The rank's part of `cfg` (whole image when world == 1)."""
    if world == 1:
        return dataclasses.replace(cfg, band_rows=cfg.height, band_stride=1, band_offset=0)
    return dataclasses.replace(cfg, band_rows=band_rows, band_stride=world, band_offset=rank)


def shard_rows(height: int, rank: int, world: int, band_rows: int = DEFAULT_BAND_ROWS) -> list[int]:
    """File rows rank `rank` renders, in output order."""
    if world == 1:
        return list(range(height))
    nb = (height + band_rows - 1) // band_rows
    return [fr for b in range(rank, nb, world) for fr in range(b * band_rows, min(height, (b + 1) * band_rows))]


_ROW_INDEX: dict = {}


def _row_index(height: int, rank: int, world: int, band_rows: int, device) -> Optional[torch.Tensor]:
    """rank's file rows as an index tensor on `device`, built once per layout: torch.tensor(list,
    device=gpu) is a blocking copy from pageable memory, which in the per-image gather would make rank 0
    wait for its own render and serialise the launches the bench keeps in flight"""
    key = (height, rank, world, band_rows, str(device))
    if key not in _ROW_INDEX:
        rows = shard_rows(height, rank, world, band_rows)
        _ROW_INDEX[key] = torch.tensor(rows, device=device) if rows else None
    return _ROW_INDEX[key]


def assemble(parts: list[torch.Tensor], height: int, band_rows: int = DEFAULT_BAND_ROWS) -> torch.Tensor:
    """Full (height, width, 3) image from the world's strips (parts[r] = rank r's strip)."""
    world = len(parts)
    if world == 1:
        return parts[0]
    width = parts[0].shape[1]
    out = parts[0].new_empty((height, width, 3))
    for r, p in enumerate(parts):
        idx = _row_index(height, r, world, band_rows, out.device)
        if idx is not None:
            out[idx] = p[: idx.shape[0]]
    return out


def gather_image(strip: torch.Tensor, cfg: RenderConfig, group=None,
                 band_rows: int = DEFAULT_BAND_ROWS) -> Optional[torch.Tensor]:
    """Gathers every rank's strip to rank 0 and returns the full image there (None elsewhere).
    Strips are padded to the largest shard so one collective moves them all."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return strip
    rows = [len(shard_rows(cfg.height, r, world, band_rows)) for r in range(world)]
    cap = max(rows)
    send = strip
    if strip.shape[0] < cap:
        send = strip.new_zeros((cap,) + tuple(strip.shape[1:]))
        send[: strip.shape[0]] = strip
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send.contiguous(), bufs, dst=0, group=group)
    if rank != 0:
        return None
    return assemble([b[:n] for b, n in zip(bufs, rows)], cfg.height, band_rows)


def render_distributed(cfg: RenderConfig, render_shard: Callable[[RenderConfig], torch.Tensor], group=None,
                       band_rows: int = DEFAULT_BAND_ROWS) -> Optional[torch.Tensor]:
    """Renders `cfg` across the process group: each rank renders its bands with
    `render_shard(shard_cfg)` (e.g. a Tracer on its own GPU) and rank 0 receives the image."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    strip = render_shard(shard_config(cfg, rank, world, band_rows))
    if world == 1:
        return strip
    return gather_image(strip, cfg, group, band_rows)


def gpu_shard_renderer(tracer, device: torch.device) -> Callable[[RenderConfig], torch.Tensor]:
    """render_shard for render_distributed: renders into a device tensor on torch's current stream."""

    def render(scfg: RenderConfig) -> torch.Tensor:
        rows = scfg.shard_rows()
        dt = torch.float64 if scfg.fp64 else torch.float32
        out = torch.empty((max(rows, 1), scfg.width, 3), dtype=dt, device=device)
        if rows:
            tracer.render_device(scfg, out.data_ptr(), torch.cuda.current_stream(device).cuda_stream)
        return out[:rows]

    return render
