#!/usr/bin/env bash
# A/B of libvpt.so builds (build_variants/libvpt_<name>.so; "base" = the in-tree libvpt.so) on one
# box: bit-exact check vs the oracle (scripts/variant_check.py), then FF + north-star MIS timing.
# usage: bash scripts/ab_var.sh name...   (BENCH_ARGS: extra bench.py flags)
set -u
mkdir -p gpurun_out
for v in "$@"; do
    lib=build_variants/libvpt_$v.so
    [ "$v" = base ] && lib=minimal_volumetric_path_tracer_amd/libvpt.so
    echo "== $v"
    VPT_LIB=$lib timeout -k 10 180 python scripts/variant_check.py > gpurun_out/chk_$v.log 2>&1
    rc=$?
    tail -3 gpurun_out/chk_$v.log
    case $rc in 0|1) ;; *) echo "STOP check rc=$rc"; exit $rc ;; esac
    VPT_LIB=$lib timeout -k 10 180 python bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$v.log; echo "STOP rc=$rc"; exit $rc; fi
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][-1]); ns=d.get('north_star') or {}; print(d['value'], 'Ms/s', d['roofline']['kernel_ms'], 'ms | MIS', ns.get('value'), ns.get('kernel_ms'))"
done
