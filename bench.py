#!/usr/bin/env python3
"""Benchmark of the hot path: Msamples/s of the volumetric radiance loop on MI355X.

Workload (BASELINE.json configs[1]): the reference's default scene (include/Sphere.cpp:11-22),
camera (src/rt.cpp:755-759) and homogeneous medium (sigma_a 0.001, sigma_s 0.009,
src/rt.cpp:794), free-flight estimator (iterativeVPTracerFree, include/vptShadeMethods.h:1263),
1024 x 1024 pixels x 256 samples per pixel.  One step = one full image: every rank renders its
row bands (interleaved 16-row bands, scaling "strong": the image is fixed, the work is split) with
one launch of pool_kernel (+ the chunk-sum reduce_kernel), then the float32 strips are gathered to
rank 0 over RCCL (N > 1).  Steps are independent images: --inflight D (default 3) keeps D of
them in flight, each on its own context and HIP stream, so that a launch's drain (the last, longest
paths of its last samples, ~0.5 ms) and its gather overlap the next launch (--inflight 1: serialized).
Inputs (the 1.4 KB scene) are resident in HBM before the timed region; nothing is skipped.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ff|mis|dense] [--no-cpu] [--inflight D]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import minimal_volumetric_path_tracer_amd as vpt  # noqa: E402
from minimal_volumetric_path_tracer_amd.distributed import gather_image  # noqa: E402

METRIC = "Msamples/s (pixels×spp/s) at 1024²; per-channel RMSE vs CPU PPM"
FLOP_PER_TEST = 20          # Sphere::intersect, include/Sphere.h:27-37
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector (= FP64 matrix) peak, spec
BAND_ROWS = 16

CONFIGS = {
    # BASELINE.json configs[1]
    "ff": dict(width=1024, height=1024, spp=256, estimator="ff", sigma_a=0.001, sigma_s=0.009),
    # BASELINE.json configs[2] (HG g = 0.5 extension), reduced to fit a quick bench: 1024 spp
    "mis": dict(width=1024, height=1024, spp=1024, estimator="mis", sigma_a=0.001, sigma_s=0.009, hg_g=0.5),
    # BASELINE.json configs[3]: dense medium, 8 bounces
    "dense": dict(width=2048, height=2048, spp=4096, estimator="ff", sigma_a=0.01, sigma_s=0.09, max_depth=8),
    # BASELINE.json configs[4]: meant for --gpus 8 (137 G samples per image; ~4 s per step on 8 GPUs)
    "mis4k": dict(width=4096, height=4096, spp=8192, estimator="mis", sigma_a=0.001, sigma_s=0.009),
}


def cpu_port_check(img: np.ndarray, c: dict, threads: int, bands: int = 12, band: int = 16) -> dict:
    """The oracle restatement (oracle/liboracle_vm.so: per-sample streams, the kernel's portable
    libm) timed on `bands` bands of `band` camera rows of the bench image, same seed and chunk
    layout, and compared with the GPU image on those rows: per-channel RMSE of the linear float32
    framebuffer (the metric's "per-channel RMSE vs CPU"; the bar is bit-exact, RMSE 0)."""
    from oracle.oracle import Oracle  # cpu_baseline leg only

    H, W, SPP = c["height"], c["width"], c["spp"]
    o = Oracle(portable=True)
    o.set_scene(vpt.default_scene())
    from minimal_volumetric_path_tracer_amd.tracer import ESTIMATORS

    est = ESTIMATORS[c["estimator"]]
    se, n, el = np.zeros(3), 0, 0.0
    for k in range(bands):
        y0 = (H - band) * k // max(bands - 1, 1)
        t = time.time()
        ref = o.render(W, H, SPP, est, sigma_a=c["sigma_a"], sigma_s=c["sigma_s"], hg_g=c.get("hg_g", 0.0),
                       max_depth=c.get("max_depth", 0), seed=0x5EED0001, y0=y0, y1=y0 + band, threads=threads)
        el += time.time() - t
        rows = slice(H - y0 - band, H - y0)  # file rows of camera rows [y0, y0 + band)
        d = img[rows].astype(np.float64) - ref[rows].astype(np.float32).astype(np.float64)
        se += (d * d).reshape(-1, 3).sum(0)
        n += band * W
    return {"value": bands * band * W * SPP / el / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle restatement (per-sample erand48 streams, portable libm), {bands} bands of {band} rows "
                      f"x {W} x {SPP} spp of the bench image, {threads} threads, {el:.1f}s",
            "rmse_vs_gpu_per_channel": [float(x) for x in np.sqrt(se / n)]}


def cpu_baseline(threads: int) -> dict:
    """The reference program itself (oracle/_ref/rt, built from /root/reference's sources by
    oracle/Makefile) on this host's cores: `rt 32` = 1024x768x32 (25 M samples, ~13 s) with its racy
    shared erand48 state, as written.  Msamples/s = w*h*spp / the elapsed time it prints
    (src/rt.cpp:824-827, includes its serial PPM write).  Falls back to the oracle restatement."""
    exe = os.path.join(ROOT, "oracle", "_ref", "rt")
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    if os.path.exists(exe):
        spp = 32
        with tempfile.TemporaryDirectory() as td:
            r = subprocess.run([exe, str(spp)], cwd=td, capture_output=True, text=True, timeout=900, env=env)
        m = re.search(r"elapsed time: ([0-9.eE+-]+)s", r.stdout)
        if r.returncode == 0 and m:
            el = float(m.group(1))
            return {"value": 1024 * 768 * spp / el / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "reference",
                    "sample": f"reference program src/rt.cpp as written (shared racy erand48 state), `rt {spp}` = "
                              f"1024x768x{spp} spp free-flight, default scene, OpenMP {threads} threads, "
                              f"elapsed {el:.2f}s incl. its PPM write"}
    from oracle.oracle import Oracle  # cpu_baseline leg only

    o = Oracle(portable=False)
    o.set_scene(vpt.default_scene())
    t = time.time()
    o.render(1024, 256, 8, 0, threads=threads)
    el = time.time() - t
    return {"value": 1024 * 256 * 8 / el / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle restatement (per-sample streams), 1024x256x8 spp free-flight, {threads} threads"}


def pmc_profile(config: str, world: int):
    """The committed rocprofv3 PMC summary of this same command for the dominant kernel
    (profiles/<round>/pmc_pool_kernel.json, scripts/pmc.sh + scripts/pmc_summary.py), newest round
    first.  Counters cannot be read live without the profiler; None when no profile matches."""
    if config != "ff" or world != 1:
        return None
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_pool_kernel.json")), reverse=True):
        try:
            return json.load(open(f))
        except (OSError, ValueError):
            continue
    return None


def pmc_traffic(prof):
    """HBM bytes per launch: (2 * FETCH_SIZE + WRITE_SIZE) * 1 KiB -- gfx950 FETCH_SIZE reports half
    of a streamed read (MI355X_MICROARCH.md, HBM)."""
    try:
        c = prof["counters"]
        return int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
    except (TypeError, KeyError):
        return None


def pmc_fp64_flop(prof):
    """All FP64 VALU work per launch, from the same profile: (add + mul + 2 fma + trans) wave
    instructions x 64 lanes x VALU lane utilisation (the FLOPS_FP64 counter is not usable on this
    stack).  Reported beside the intersection-only roofline of SURVEY 8(d)."""
    try:
        c = prof["counters"]
        ops = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + 2 * c["SQ_INSTS_VALU_FMA_F64"] + \
            c["SQ_INSTS_VALU_TRANS_F64"]
        return ops * 64 * prof["derived"]["valu_lane_utilization"]
    except (TypeError, KeyError):
        return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="ff", choices=list(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--chunk", type=int, default=0, help="samples per work unit (0 = auto: 32, more above 4096 spp, tapered; vpt_chunks.h)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="steps in flight: each on its own context + HIP stream, so one launch's drain (its "
                         "last, longest paths) overlaps the next launch's start; 1 = strictly serialized")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    c = CONFIGS[args.config]
    H, W, SPP = c["height"], c["width"], c["spp"]
    band = BAND_ROWS if world > 1 else H
    if world > 1 and H % (band * world):
        raise SystemExit("image height must be a multiple of 16 * world size")
    cfg = vpt.RenderConfig(**c, seed=0x5EED0001, band_rows=band, band_stride=world, band_offset=rank,
                           chunk_spp=args.chunk)
    D = max(1, args.inflight)
    tracers = [vpt.Tracer(dev.index) for _ in range(D)]  # one context (work queue, partials) per slot
    tracer = tracers[0]
    rows = cfg.shard_rows()
    outs = [torch.empty((rows, W, 3), dtype=torch.float32, device=dev) for _ in range(D)]
    images = [torch.empty((H, W, 3), dtype=torch.float32, device=dev) if rank == 0 else None for _ in range(D)]
    streams = [torch.cuda.current_stream(dev)] if D == 1 else [torch.cuda.Stream(dev) for _ in range(D)]
    stream = streams[0]

    # ray-sphere tests per sample of the reference algorithm on this workload (counting build of
    # the same kernel, untimed; 1/16 of the spp -- the per-sample mean is what is needed)
    cnt_cfg = vpt.RenderConfig(**{**c, "spp": max(1, SPP // 16)}, seed=0x5EED0001, band_rows=band,
                               band_stride=world, band_offset=rank)
    tests, iters = tracer.count_work(cnt_cfg)
    T = tests / (rows * W * cnt_cfg.spp)

    def step(k, ev=None):
        """step k: the whole image on slot k % D -- render the rank's bands, then (N > 1) the RCCL
        gather of the strips to rank 0, all on the slot's stream (the gather of step k overlaps the
        render of step k + 1 on the next slot)"""
        j = k % D
        s = streams[j]
        with torch.cuda.stream(s):
            if ev is not None:
                ev[0].record(s)
            tracers[j].render_device(cfg, outs[j].data_ptr(), s.cuda_stream)
            if ev is not None:
                ev[1].record(s)
            if world > 1:
                full = gather_image(outs[j], cfg, band_rows=band)  # RCCL gather of the strips to rank 0
                if rank == 0:
                    images[j].copy_(full)
            elif rank == 0:
                images[j].copy_(outs[j])

    for k in range(max(args.warmup, D if args.warmup else 0)):
        step(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, evs[k] if D == 1 else None)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if D > 1:
        # overlapping launches make per-launch events meaningless: the kernel's duration for the
        # roofline comes from serialized launches of the same render, on one stream, right after
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(min(max(args.steps, 2), 5))]
        for a, b in evs:
            a.record(stream)
            tracer.render_device(cfg, outs[0].data_ptr(), stream.cuda_stream)
            b.record(stream)
        torch.cuda.synchronize(dev)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_step = H * W * SPP
    value = samples_step * args.steps / elapsed / 1e6
    launch_samples = rows * W * SPP
    achieved = launch_samples * FLOP_PER_TEST * T / (kern_ms * 1e-3) / 1e12
    prof = pmc_profile(args.config, world)
    full = pmc_fp64_flop(prof)
    if rank == 0:
        for j in range(1, min(D, args.steps)):  # every slot rendered the same image
            assert torch.equal(images[j], images[0]), "in-flight slots disagree"
        img = images[0].float().cpu().numpy()
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: the reference's default scene/camera/medium, per-sample erand48 streams (seed 0x5EED0001)",
            "config": {
                "workload": f"{c['estimator']} {W}x{H}x{SPP}spp default scene, sigma_a {c['sigma_a']} sigma_s {c['sigma_s']}"
                            + (f", HG g {c['hg_g']}" if c.get("hg_g") else "") + (f", max depth {c['max_depth']}" if c.get("max_depth") else ""),
                "width": W, "height": H, "spp": SPP, "estimator": c["estimator"],
                "parallelism": f"row bands of {band} interleaved over {world} GPU(s), RCCL gather to rank 0" if world > 1
                else "1 GPU",
                "inflight": D,
            },
            "roofline": {
                "bound": "mfma",
                "achieved": round(achieved, 4),
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP64_PEAK_TFLOPS, 5),
                "traffic": pmc_traffic(prof),
                "kernel": f"pool_kernel<{'FF' if c['estimator'] == 'ff' else 'MIS'}> + reduce_kernel (one launch pair)",
                "kernel_ms": round(kern_ms, 3),
                "kernel_ms_from": "HIP events around each launch of the timed steps on their stream" if D == 1 else
                                  f"HIP events around {len(evs)} serialized launches of the same render on one stream, "
                                  f"right after the timed region (its {D} in-flight steps overlap)",
                "algorithmic": f"{FLOP_PER_TEST} FP64 flop x {T:.2f} ray-sphere tests per sample (SURVEY 8d) x "
                               f"{launch_samples} samples per launch",
                "all_fp64_tflops": round(full / (kern_ms * 1e-3) / 1e12, 3) if full else None,
                "all_fp64_frac": round(full / (kern_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4) if full else None,
                "note": "FP64 compute roof: MI355X FP64 vector and FP64 matrix peaks are both 78.6 TFLOP/s (spec); "
                        "the kernel runs on the FP64 VALU, no MFMA (no dense contraction exists). achieved/frac "
                        "count intersection flops only (SURVEY 8d); all_fp64_* count every FP64 VALU op of the "
                        "kernel (committed PMC profile of this command, profiles/r*/pmc_pool_kernel.json)",
            },
            "image_mean": [round(float(x), 6) for x in img.reshape(-1, 3).mean(0)],
        }
        if world == 1 and not args.no_cpu:
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
            res["cpu_baseline"] = cpu_baseline(threads)
            # the per-thread-RNG flavour + the per-channel RMSE of sampled rows vs the GPU image
            res["cpu_baseline"]["port_per_sample_rng"] = cpu_port_check(img, c, threads)
        print(json.dumps(res))
    for t in tracers:
        t.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
