set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b_d3.log 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --inflight 2 > gpurun_out/b_d2.log 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --inflight 1 > gpurun_out/b_d1.log 2>&1
for f in b_d3 b_d2 b_d1; do grep '^{' gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['image_mean'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d3 -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_d3.log 2>&1
find gpurun_out/prof_d3 -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-200 | head -5
grep '^{' gpurun_out/prof_d3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('prof run', d['value'], d['roofline']['kernel_ms'])"
