set -u
export TMPDIR=/tmp
bash scripts/gpu_check.sh r06r tests smoke || exit $?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
REPS=2 CFGS="ff march pt" bash scripts/ab.sh r06r old base || exit $?
echo "== end $(date +%T)"
