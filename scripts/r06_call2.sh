set -u
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r06c.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_r06c.log; echo "tests rc=$rc"
case $rc in 0|1) ;; *) echo STOP; exit $rc ;; esac
echo "== ab $(date +%T)"
NOCHECK=1 REPS=3 bash scripts/ab.sh r06b base e3 nodiv noacos allsel || exit $?
echo "== end $(date +%T)"
