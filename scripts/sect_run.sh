#!/usr/bin/env bash
# Section-timer profile (debug build with -DVPT_SECTIONS=1) of FF configs[1] and MIS + HG configs[2]
# shares.  usage: bash scripts/sect_run.sh <tag> <variant name>
set -u
OUT=gpurun_out/sect_$1
mkdir -p "$OUT"
for est in ff mis; do
    VPT_LIB=build_variants/libvpt_$2.so timeout -k 10 240 python scripts/sect_stats.py $est > "$OUT/$est.txt" 2>&1
    rc=$?; cat "$OUT/$est.txt"; [ $rc -eq 0 ] || { echo "STOP sect rc=$rc"; exit $rc; }
done
