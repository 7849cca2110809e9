set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "isect_sqrt or device_math or inv_sqrt or trace_batch or render" > gpurun_out/pytest_r06k.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r06k.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash scripts/ab.sh r06k old base || exit $?
echo "== end $(date +%T)"
