#!/usr/bin/env bash
# Round-4 GPU call: parity tests, then an A/B of library builds (VPT_LIB) on FF configs[1] and the
# north-star configs[2], serialized launches.  Each step under its own time limit; stops at the first failure.
# usage: bash scripts/gpu_r04.sh <tag> [tests|notests] lib1.so lib2.so ...
set -u
TAG=$1; shift
MODE=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$MODE" = tests ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
        > "$OUT/tests.log" 2>&1
    rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || { echo "STOP tests rc=$rc"; exit $rc; }
fi
for rep in 1 2; do
    for L in "$@"; do
        VPT_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --inflight 1 > "$OUT/ab.log" 2>&1
        rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/ab.log"; echo "STOP bench rc=$rc"; exit $rc; }
        python - "$OUT/ab.log" "$L" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ns = d.get("north_star") or {}
print(f"{sys.argv[2]:55s} FF {d['value']:.1f} Ms/s kernel {d['roofline']['kernel_ms']:.3f} ms | "
      f"MIS+HG {ns.get('value', 0):.1f} Ms/s kernel {ns.get('kernel_ms', 0):.2f} ms | build {d.get('build_id')}")
PY
    done
done
