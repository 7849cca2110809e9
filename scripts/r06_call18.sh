set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06n base au || exit $?
echo "== end $(date +%T)"
