#!/usr/bin/env bash
# Quick GPU iteration: parity tests (bit-exact vs the oracle), then the FF bench line without the
# CPU leg and the north-star config.  Each step under its own time limit; stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || { echo "STOP tests rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-north-star ${BENCH_ARGS:-} > gpurun_out/quick_bench.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/quick_bench.log; echo "STOP bench rc=$rc"; exit $rc; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/quick_bench.log') if l.startswith('{')][-1]); print('FF', d['value'], 'Ms/s', d['roofline']['kernel_ms'], 'ms frac', d['roofline']['frac'], d['image_mean'])"
