#!/usr/bin/env bash
# PC sampling probe of one bench step (rocprofv3 --pc-sampling-*, no counters).
# usage: bash scripts/pcsamp.sh <tag> [method] [unit] [interval] [bench args...]
set -u
TAG=${1:-probe}; METHOD=${2:-stochastic}; UNIT=${3:-cycles}; IV=${4:-65536}
shift 4 2>/dev/null || shift $#
ARGS=${*:---steps 1 --warmup 0 --no-cpu --no-north-star --inflight 1}
OUT=gpurun_out/pcs_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/list.txt" 2>&1; echo "list rc=$?"
grep -i -A12 "pc.sampl\|PC_SAMPL" "$OUT/list.txt" | head -60
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method "$METHOD" --pc-sampling-unit "$UNIT" \
    --pc-sampling-interval "$IV" -d "$OUT/run" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/run.log" 2>&1
rc=$?
echo "pcs rc=$rc"; tail -5 "$OUT/run.log"
find "$OUT/run" -type f | head; exit $rc
