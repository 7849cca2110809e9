#!/usr/bin/env bash
# A/B of libvpt.so builds on other bench configs (kernel ms per step, serialized launches).
# usage: CFGS="march pt" REPS=2 bash scripts/ab_cfg.sh <tag> name...   ("base" = the in-tree libvpt.so)
set -u
TAG=$1; shift
OUT=gpurun_out/abcfg_$TAG
mkdir -p $OUT
for rep in $(seq 1 "${REPS:-2}"); do
for v in "$@"; do
  L=minimal_volumetric_path_tracer_amd/libvpt.so; [ $v = base ] || L=build_variants/libvpt_$v.so
  for c in ${CFGS:-march pt dense}; do
    VPT_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu --inflight 1 > $OUT/${v}_$c.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -3 $OUT/${v}_$c.log; echo STOP $rc; exit $rc; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" $OUT/${v}_$c.log $v $c
  done
done
done
