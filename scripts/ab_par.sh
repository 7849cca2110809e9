#!/usr/bin/env bash
# GPU parity tests against one A/B variant, then timing of several (scripts/ab.sh)
# usage: bash scripts/ab_par.sh <variant .so for the parity run> "ENV=.." ...
set -u
v=$1; shift
VPT_LIB=$v timeout -k 10 150 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/ab_pytest.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; grep -m5 -E "Error|assert" gpurun_out/ab_pytest.log; exit $rc; fi
bash scripts/ab.sh "$@"
