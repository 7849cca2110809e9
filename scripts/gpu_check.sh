#!/usr/bin/env bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.  Each GPU step has its own
# time limit; a fault, abort, segfault or time-out ends the script (no further GPU work).
# Usage (on the GPU box, from the repo root):  bash scripts/gpu_check.sh [tag] [steps...]
#   steps: tests smoke bench prof pmc   (default: tests smoke bench prof)
# Profiles run bench.py --inflight 1: with overlapping launches (the default --inflight 3) each
# dispatch's begin-end span includes time spent waiting for the other launches' workgroups.
set -u
TAG=${1:-r01}
shift || true
STEPS=${*:-tests smoke bench prof}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    case $rc in
        124|137|134|139|-6|-11) echo "STOP: $name ended with $rc"; exit $rc ;;
    esac
    return 0
}

for s in $STEPS; do
    case $s in
        tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py --steps 3 --warmup 1 ;;
        prof)  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- \
                   python3 bench.py --steps 3 --warmup 1 --no-cpu --inflight 1 ;;
        pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$TAG" -o run --output-format csv -- \
                   python3 bench.py --steps 1 --warmup 0 --no-cpu --inflight 1 &&
               run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$TAG" -o run --output-format csv -- \
                   python3 bench.py --steps 1 --warmup 0 --no-cpu --inflight 1 ;;
        *) echo "unknown step $s" ;;
    esac
done
echo "== done"
