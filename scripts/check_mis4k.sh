set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 170 python bench.py --config mis4k --steps 1 --warmup 0 --inflight 1 --no-cpu > gpurun_out/bench_mis4k.log 2>&1
grep '^{' gpurun_out/bench_mis4k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mis4k', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['image_mean'])"
