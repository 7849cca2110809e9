#!/usr/bin/env bash
# A/B of libvpt.so builds on one box: bit-exact check of each variant vs the oracle
# (scripts/variant_check.py), then REPS interleaved rounds of FF configs[1] + north-star configs[2]
# kernel timings (serialized launches).  "base" = the in-tree libvpt.so.
# usage: REPS=2 bash scripts/ab2.sh <tag> name...
set -u
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
lib() { if [ "$1" = base ]; then echo minimal_volumetric_path_tracer_amd/libvpt.so; else echo build_variants/libvpt_$1.so; fi; }
for v in "$@"; do
    VPT_LIB=$(lib "$v") timeout -k 10 240 python scripts/variant_check.py > "$OUT/chk_$v.log" 2>&1
    rc=$?
    echo "check $v rc=$rc: $(tail -1 "$OUT/chk_$v.log")"
    case $rc in 0|1) ;; *) echo "STOP check rc=$rc"; exit $rc ;; esac
done
for rep in $(seq 1 "${REPS:-2}"); do
    for v in "$@"; do
        VPT_LIB=$(lib "$v") timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --inflight 1 ${BENCH_ARGS:-} \
            > "$OUT/b_$v.log" 2>&1
        rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_$v.log"; echo "STOP bench rc=$rc"; exit $rc; }
        python - "$OUT/b_$v.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ns = d.get("north_star") or {}
print(f"{sys.argv[2]:12s} FF kernel {d['roofline']['kernel_ms']:.3f} ms | MIS+HG kernel {ns.get('kernel_ms', 0):.2f} ms")
PY
    done
done
