#!/usr/bin/env bash
# A/B timing of libvpt.so builds (build_variants/libvpt_<name>.so, scripts/build_variant.sh) on one
# box, one process per variant: Msamples/s and kernel ms of the default bench config, plus the
# estimator-4 pool render vs the oracle (scripts/dbg_e4b.py).  usage: bash scripts/ab_lib.sh name...
set -u
mkdir -p gpurun_out
for v in "$@"; do
    lib=build_variants/libvpt_$v.so
    [ "$v" = base ] && lib=minimal_volumetric_path_tracer_amd/libvpt.so
    echo "== $v"
    VPT_LIB=$lib timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab.log; echo "STOP rc=$rc"; exit $rc; fi
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab.log') if l.startswith('{')][-1]); ns=d.get('north_star') or {}; print(d['value'], 'Ms/s', d['roofline']['kernel_ms'], 'ms', d['image_mean'], '| MIS', ns.get('value'), ns.get('kernel_ms'))"
    if [ -n "${AB_CHECK:-}" ]; then VPT_LIB=$lib timeout -k 10 120 python scripts/dbg_e4b.py || exit 1; fi
done
