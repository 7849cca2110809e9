set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06z base fsd fmr fmc || exit $?
echo "== end $(date +%T)"
