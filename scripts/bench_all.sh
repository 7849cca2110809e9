# bench.py on the three single-GPU configs (ff with the CPU baseline, mis, dense); logs under gpurun_out/
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1
grep '^{' gpurun_out/bench_full.log
timeout -k 10 300 python bench.py --config mis --no-cpu > gpurun_out/bench_mis.log 2>&1
grep '^{' gpurun_out/bench_mis.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mis', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --config dense --no-cpu --steps 2 > gpurun_out/bench_dense.log 2>&1
grep '^{' gpurun_out/bench_dense.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dense', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
