set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "chunk or handout" > gpurun_out/pt_chunk.log 2>&1
tail -2 gpurun_out/pt_chunk.log
timeout -k 10 200 python -u scripts/shard_time.py ff 1 2 4 8 > gpurun_out/shard_taper.log 2>&1
cat gpurun_out/shard_taper.log
CHUNK=32 timeout -k 10 200 python -u scripts/shard_time.py ff 1 2 4 8 > gpurun_out/shard_uni.log 2>&1
cat gpurun_out/shard_uni.log
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_taper.log 2>&1
grep '^{' gpurun_out/bench_taper.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])"
