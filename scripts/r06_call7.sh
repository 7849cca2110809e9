set -u
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r06f.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_r06f.log; echo "tests rc=$rc"
case $rc in 0|1) ;; *) echo STOP; exit $rc ;; esac
echo "== dup $(date +%T)"
bash scripts/dup_pmc.sh r06b base base2 dup1 dup2 dup3 dup4 dup5 dup6 dup7 dup8 dup9 dup10 dup11 dup12 dup13 dup14 dup15 dup16
echo "== end $(date +%T)"
