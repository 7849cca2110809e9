set -u
export TMPDIR=/tmp
echo "== probe $(date +%T)"
VPT_LIB=build_variants/libvpt_athalf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "atan2 or dir_trig or device_math_bitwise or hg" > gpurun_out/pytest_probe_r06g.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|differ" gpurun_out/pytest_probe_r06g.log | tail -8; echo "probe rc=$rc"
case $rc in 0|1) ;; *) echo STOP; exit $rc ;; esac
REPS=3 bash scripts/ab.sh r06f base at athalf g4 tries2 tries4 scheddef minreg || exit $?
echo "== end $(date +%T)"
