#!/usr/bin/env bash
# One GPU call for a round's final measurement of the in-tree build: parity tests, smoke, bench,
# rocprofv3 kernel trace, PMC passes + their summaries (copied over profiles/<round>/pmc_pool_kernel*.json
# on the box, so that a second bench run carries the PMC fields), that bench, and the shard-scaling
# projection.  Every GPU step has its own time limit; any failure ends the script.
# usage: bash scripts/final_run.sh <tag> <round dir, e.g. r04>
set -u
TAG=$1; RD=$2
OUT=gpurun_out
bash scripts/gpu_check.sh "$TAG" tests smoke bench prof || exit $?
bash scripts/pmc.sh "$TAG" || exit $?
python3 scripts/pmc_summary.py "$OUT/pmc_$TAG" 'pool_kernel<0, false>' > "$OUT/pmc_pool_kernel_$TAG.json" || exit 1
python3 scripts/pmc_summary.py "$OUT/pmc_$TAG" 'pool_kernel<1, false>' > "$OUT/pmc_pool_kernel_mis_$TAG.json" || exit 1
cp "$OUT/pmc_pool_kernel_$TAG.json" "profiles/$RD/pmc_pool_kernel.json"
cp "$OUT/pmc_pool_kernel_mis_$TAG.json" "profiles/$RD/pmc_pool_kernel_mis.json"
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > "$OUT/bench_$TAG.log" 2>&1 || { echo "STOP bench2"; exit 1; }
grep '^{' "$OUT/bench_$TAG.log" | tail -1
bash scripts/gpu_pipe.sh "$TAG" || exit $?
echo "== final done"
