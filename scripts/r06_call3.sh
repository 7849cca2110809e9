set -u
export TMPDIR=/tmp
echo "== probe tests (in-tree build) $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "inv_sqrt or dir_trig_cone or shared_reciprocal or device_math_bitwise" > gpurun_out/pytest_probe_r06d.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|differ" gpurun_out/pytest_probe_r06d.log | tail -12; echo "probe rc=$rc"
case $rc in 0|1) ;; *) echo STOP; exit $rc ;; esac
for v in base vnone e3 vseed vacos vdiv allsel; do
    lib=minimal_volumetric_path_tracer_amd/libvpt.so
    [ $v = base ] || lib=build_variants/libvpt_$v.so
    VPT_LIB=$lib timeout -k 10 300 python scripts/variant_check.py > gpurun_out/chk_$v.log 2>&1
    rc=$?; echo "check $v rc=$rc: $(tail -3 gpurun_out/chk_$v.log | tr '\n' ' ')"
    case $rc in 0|1) ;; *) echo STOP; exit $rc ;; esac
done
echo "== end $(date +%T)"
