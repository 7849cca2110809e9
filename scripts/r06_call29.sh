#!/usr/bin/env bash
# Round 6 final measurement of the shipped build: tests, smoke, bench, rocprof, PMC, bench with PMC fields,
# shard projection (final_run.sh), then wait attribution, section timers and the per-section DUP counts.
set -u
bash scripts/final_run.sh r06final4 r06 || exit $?
bash scripts/wait_attrib.sh r06w4 || exit $?
bash scripts/sect_run.sh r06s4 sect || exit $?
bash scripts/dup_pmc.sh r06e base dup1 dup2 dup3 dup4 dup5 dup6 dup7 dup8 dup9 dup10 dup11 dup12 dup13 dup14 dup15 dup16 || exit $?
python3 scripts/dup_summary.py gpurun_out/dup_r06e > gpurun_out/dup_r06e/summary.txt || exit 1
echo "== call29 done"
