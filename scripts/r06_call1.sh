set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests (e3 build) $(date +%T)"
VPT_LIB=build_variants/libvpt_e3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r06b.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu_r06b.log; echo "tests rc=$rc"
case $rc in 0|1) ;; *) echo STOP; exit $rc ;; esac
echo "== ab e3 $(date +%T)"
NOCHECK=1 REPS=2 bash scripts/ab.sh r06e3 base e3 || exit $?
echo "== dup $(date +%T)"
bash scripts/dup_pmc.sh r06 base base2 dup1 dup2 dup3 dup4 dup5 dup6 dup7 dup8 dup9 dup10 dup11 dup12 dup13 dup14 dup15 dup16
echo "== end $(date +%T)"
