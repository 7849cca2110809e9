#!/usr/bin/env bash
# The one A/B driver: libvpt.so builds compared on one GPU box.
#   1. bit-exact check of every variant vs the oracle (scripts/variant_check.py: 11 scenes x 6
#      estimators, the pool renders of configs[1]-style layouts), a failing variant stops the run;
#   2. REPS interleaved rounds of kernel timings (serialized launches, bench.py --inflight 1) of
#      FF configs[1] + the north-star configs[2] (MIS + HG), or of the configs named in CFGS.
# Variants: "base" = the in-tree minimal_volumetric_path_tracer_amd/libvpt.so, any other name =
# build_variants/libvpt_<name>.so (scripts/build_variant.sh <name> [flags]).  Every DESIGN.md A/B row
# of round 5 on quotes this command.
# usage: [REPS=2] [CFGS="ff march pt dense"] [NOCHECK=1] bash scripts/ab.sh <tag> name...
set -u
TAG=${1:?tag}; shift
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
lib() { if [ "$1" = base ]; then echo minimal_volumetric_path_tracer_amd/libvpt.so; else echo build_variants/libvpt_$1.so; fi; }
for v in "$@"; do  # every variant built before any GPU work
    [ -f "$(lib "$v")" ] || { echo "STOP: $(lib "$v") is missing (scripts/build_variant.sh $v ...)"; exit 2; }
done
if [ -z "${NOCHECK:-}" ]; then
    for v in "$@"; do
        VPT_LIB=$(lib "$v") timeout -k 10 240 python scripts/variant_check.py > "$OUT/chk_$v.log" 2>&1
        rc=$?
        echo "check $v rc=$rc: $(tail -1 "$OUT/chk_$v.log")"
        case $rc in 0) ;; *) echo "STOP check rc=$rc"; exit 3 ;; esac
    done
fi
for rep in $(seq 1 "${REPS:-2}"); do
    for v in "$@"; do
        for c in ${CFGS:-ff}; do
            VPT_LIB=$(lib "$v") timeout -k 10 300 python bench.py --config "$c" --steps 3 --warmup 1 --no-cpu --inflight 1 \
                ${BENCH_ARGS:-} > "$OUT/b_${v}_$c.log" 2>&1
            rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${v}_$c.log"; echo "STOP bench rc=$rc"; exit $rc; }
            python - "$OUT/b_${v}_$c.log" "$v" "$c" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ns = d.get("north_star") or {}
extra = f" | MIS+HG kernel {ns['kernel_ms']:.2f} ms" if ns else ""
print(f"{sys.argv[2]:14s} {sys.argv[3]:6s} kernel {d['roofline']['kernel_ms']:.3f} ms, {d['value']:.1f} Ms/s{extra}")
PY
        done
    done
done
