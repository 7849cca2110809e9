#!/usr/bin/env bash
# A/B timing of kernel variants selected by environment (one process per variant, same box).
# usage: bash scripts/ab.sh "ENV=.. ENV2=.." "ENV=.." ...
set -u
mkdir -p gpurun_out
for v in "$@"; do
    echo "== $v"
    env $v timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab.log; echo "STOP rc=$rc"; exit $rc; fi
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab.log') if l.startswith('{')][-1]); print(d['value'], 'Ms/s', d['roofline']['kernel_ms'], 'ms', d['image_mean'])"
done
