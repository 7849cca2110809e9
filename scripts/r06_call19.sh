set -u
export TMPDIR=/tmp
VPT_LIB=build_variants/libvpt_zr.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "isect_sqrt" > gpurun_out/pytest_r06o.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r06o.log; [ $rc -eq 0 ] || exit $rc
REPS=2 CFGS="ff march pt" bash scripts/ab.sh r06o base zr zrm || exit $?
echo "== end $(date +%T)"
