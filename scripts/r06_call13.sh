set -u
export TMPDIR=/tmp
bash scripts/gpu_check.sh r06j tests smoke || exit $?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
REPS=2 bash scripts/ab.sh r06j old base || exit $?
echo "== end $(date +%T)"
