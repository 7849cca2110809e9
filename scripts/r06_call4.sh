set -u
export TMPDIR=/tmp
echo "== probe tests (in-tree build) $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "inv_sqrt or dir_trig_cone or shared_reciprocal or device_math_bitwise or sqrt" > gpurun_out/pytest_probe_r06e.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|differ" gpurun_out/pytest_probe_r06e.log | tail -12; echo "probe rc=$rc"
case $rc in 0|1) ;; *) echo STOP; exit $rc ;; esac
REPS=3 bash scripts/ab.sh r06c base nobf nodiv nosel || exit $?
echo "== end $(date +%T)"
