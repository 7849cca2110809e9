"""bench.py --gpus N without a launcher (Missing #1): the bench starts N rank processes
itself and never runs on fewer GPUs than asked.  CPU tests of the launch logic (bench.launch_ranks,
the renderer mocked by tests/rank_probe.py, gloo) and of the refusals; the one-GPU box checks the
same refusal and the real renderer + gather in tests/test_gpu_multiproc.py."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tests", "rank_probe.py")


def _bench():
    sys.path.insert(0, ROOT)
    import bench

    return bench


@pytest.mark.parametrize("n", [2, 3])
def test_launch_ranks_starts_n_ranks_that_see_world_n(tmp_path, n):
    bench = _bench()
    out = tmp_path / "r.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    rc = bench.launch_ranks(n, [sys.executable, PROBE, str(out)], env=env, timeout=180)
    assert rc == 0
    r = json.load(open(out))
    assert r["world"] == n
    assert [s["rank"] for s in r["seen"]] == list(range(n))
    assert all(s["world"] == n and s["local"] == str(s["rank"]) and s["master"] == "127.0.0.1" for s in r["seen"])
    assert r["image"] == [float(i) for i in range(48)]  # every file row from the rank that owns it


def test_launch_ranks_fails_when_a_rank_fails(tmp_path):
    bench = _bench()
    rc = bench.launch_ranks(2, [sys.executable, PROBE, str(tmp_path / "r.json"), "fail-rank-1"], timeout=120)
    assert rc == 3  # rank 1's status; rank 0 (sleeping) was stopped, not waited out
    assert not (tmp_path / "r.json").exists()


def _run_bench(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=180, env=env, cwd=ROOT)


def test_bench_refuses_more_gpus_than_the_node_has():
    """here there is no GPU: --gpus 2 must exit non-zero before any rank starts, never render on one"""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("node has >= 2 GPUs")
    r = _run_bench(["--gpus", "2", "--no-cpu"])
    assert r.returncode == 2, r.stderr[-500:]
    assert "refusing to run on fewer" in r.stderr
    assert not r.stdout.strip()


def test_bench_refuses_world_size_mismatch():
    r = _run_bench(["--gpus", "2", "--no-cpu"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
    r = _run_bench(["--gpus", "1", "--no-cpu"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_bench_shared_device_needs_gloo():
    r = _run_bench(["--gpus", "2", "--shared-device"])
    assert r.returncode != 0 and "gloo" in r.stderr
