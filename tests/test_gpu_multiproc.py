"""Several processes on the one-GPU box (Missing #2): the real renderer (libvpt) in 2 and 3
rank processes that share cuda:0, their strips gathered over gloo, and bench.py's N > 1 branch (gather
inside the timed step, max over ranks of the elapsed time) driven the same way.  The gathered image
must equal the single-process render bit for bit: every pixel's samples are summed once, in order,
by whichever rank owns its row (src/rt.cpp:786-800).  The 8-GPU RCCL run itself is the driver's."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
from conftest import bitwise_equal

import minimal_volumetric_path_tracer_amd as vpt

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _clean_env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}


@pytest.mark.parametrize("world,est,g,band", [(2, "ff", 0.0, 16), (3, "ff", 0.0, 16), (2, "mis", 0.5, 16),
                                              (3, "mis", 0.5, 8)])
def test_libvpt_shards_gathered_over_processes(gpu_tracer, tmp_path, world, est, g, band):
    sys.path.insert(0, ROOT)
    import bench

    W, H, SPP = 64, 48, 8
    out = tmp_path / "img.npy"
    rc = bench.launch_ranks(world, [sys.executable, os.path.join(ROOT, "tests", "gpu_rank_worker.py"), str(out), est,
                                    str(W), str(H), str(SPP), repr(g), str(band)], env=_clean_env(), timeout=150)
    assert rc == 0
    img = np.load(out)
    gpu_tracer.set_scene(vpt.default_scene())
    ref = gpu_tracer.render(vpt.RenderConfig(width=W, height=H, spp=SPP, estimator=est, hg_g=g, seed=0x5EED0001))
    assert img.shape == ref.shape == (H, W, 3)
    assert bitwise_equal(img, ref).all()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_multi_rank_branch(gpu_tracer, tmp_path, world):
    """bench.py --gpus N on one GPU with --shared-device --dist-backend gloo: N ranks, the strips gathered
    inside the timed steps, the job's elapsed time = the max over ranks; the saved image equals the
    single-process render bit for bit"""
    W, H, SPP = 64, 96, 8
    out = tmp_path / "bench.npy"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dist-backend", "gloo",
                        "--shared-device", "--size", f"{W}x{H}x{SPP}", "--no-cpu", "--no-north-star", "--inflight", "2",
                        "--steps", "3", "--warmup", "1", "--save-image", str(out)],
                       capture_output=True, text=True, timeout=170, env=_clean_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints the line
    res = json.loads(lines[0])
    pg = res["config"]["process_group"]
    assert res["n_gpus"] == world and pg["world_size"] == world and pg["backend"] == "gloo"
    assert len(pg["rank_devices"]) == world and all(d.startswith(f"rank {k}: cuda:0") for k, d in enumerate(pg["rank_devices"]))
    assert len(pg["rank_elapsed_s"]) == world
    # the N > 1 diagnostics: every rank's serialized kernel time and rank 0's gather time
    assert len(pg["rank_kernel_ms"]) == world and all(k > 0 for k in pg["rank_kernel_ms"])
    assert pg["gather_ms"] is not None and pg["gather_ms"] >= 0
    # ms_per_step comes from the max-reduced elapsed time
    assert res["ms_per_step"] == pytest.approx(max(pg["rank_elapsed_s"]) / 3 * 1e3, abs=2e-3)
    gpu_tracer.set_scene(vpt.default_scene())
    ref = gpu_tracer.render(vpt.RenderConfig(width=W, height=H, spp=SPP, estimator="ff", seed=0x5EED0001))
    assert bitwise_equal(np.load(out), ref).all()


def test_bench_refuses_more_gpus_than_the_box_has():
    """--gpus 2 on the one-GPU box: non-zero exit with a clear message, never a one-GPU line"""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("box has >= 2 GPUs")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu"], capture_output=True,
                       text=True, timeout=120, env=_clean_env(), cwd=ROOT)
    assert r.returncode == 2 and "refusing to run on fewer" in r.stderr, r.stderr[-500:]
    assert not r.stdout.strip()


def test_assemble_does_not_block_the_host():
    """rank 0's per-image reassembly (distributed.assemble, inside bench.py's timed step) enqueues device
    work only: a blocking host copy there would make rank 0 wait for its own render and serialise the
    launches the bench keeps in flight (the RCCL runs of the driver's scaling bench go through it)"""
    import time

    import torch

    from minimal_volumetric_path_tracer_amd.distributed import assemble, shard_rows

    dev = torch.device("cuda:0")
    H, W, world = 64, 32, 4
    parts = [torch.full((len(shard_rows(H, r, world)), W, 3), float(r), device=dev) for r in range(world)]
    first = assemble(parts, H)  # builds the per-layout row indices (once)
    torch.cuda.synchronize()
    for r in range(world):
        assert bool((first[torch.tensor(shard_rows(H, r, world), device=dev)] == r).all())
    # non-blocking checked directly, not by a wall-clock ratio: with ~0.1 s of device time
    # queued ahead, assemble() returns while an event recorded behind that work is still pending, and
    # it makes no host-device round trip (torch.cuda.synchronize and host copies would raise)
    torch.cuda._sleep(200_000_000)
    queued = torch.cuda.Event()
    queued.record()
    real_sync, real_tensor = torch.cuda.synchronize, torch.tensor

    def no_sync(*a, **k):
        raise AssertionError("assemble() synchronised the device")

    def no_host_tensor(data, *a, device=None, **k):
        if device is not None and torch.device(device).type == "cuda":
            raise AssertionError("assemble() copied host data to the device")
        return real_tensor(data, *a, device=device, **k)

    torch.cuda.synchronize, torch.tensor = no_sync, no_host_tensor
    try:
        out = assemble(parts, H)
        pending = not queued.query()
    finally:
        torch.cuda.synchronize, torch.tensor = real_sync, real_tensor
    assert pending, "the queued device work finished before assemble() returned"
    torch.cuda.synchronize()
    assert torch.equal(out, first)
