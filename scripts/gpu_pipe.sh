#!/usr/bin/env bash
# Strong-scaling projection from one GPU: rank 0's 1/N row-band shard rendered back to back,
# serialized (depth 1) and 3 in flight, for FF configs[1] and MIS + HG configs[2].
# usage: bash scripts/gpu_pipe.sh <tag>
set -u
OUT=gpurun_out/pipe_$1
mkdir -p "$OUT"
DEPTHS=1,3 STEPS=12 timeout -k 10 300 python -u scripts/pipe_time.py ff 1 2 4 8 > "$OUT/pipe_ff.txt" 2>&1
rc=$?; cat "$OUT/pipe_ff.txt"; [ $rc -eq 0 ] || { echo "STOP rc=$rc"; exit $rc; }
DEPTHS=1,3 STEPS=6 timeout -k 10 400 python -u scripts/pipe_time.py mis 1 2 4 8 > "$OUT/pipe_mis.txt" 2>&1
rc=$?; cat "$OUT/pipe_mis.txt"; [ $rc -eq 0 ] || { echo "STOP rc=$rc"; exit $rc; }
