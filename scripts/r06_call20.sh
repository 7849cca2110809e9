set -u
export TMPDIR=/tmp
VPT_LIB=build_variants/libvpt_zr2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "isect_sqrt or march or punctual or surface_pt or e5 or e789" > gpurun_out/pytest_r06p.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r06p.log; [ $rc -eq 0 ] || exit $rc
REPS=2 CFGS="ff march pt" bash scripts/ab.sh r06p base zr2 || exit $?
echo "== end $(date +%T)"
