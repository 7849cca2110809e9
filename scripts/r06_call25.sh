set -u
export TMPDIR=/tmp
bash scripts/gpu_check.sh r06t tests smoke || exit $?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
REPS=2 bash scripts/ab.sh r06t old base || exit $?
echo "== end $(date +%T)"
