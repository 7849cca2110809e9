set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06h base fc0 fc1 fc2 fc1nr || exit $?
echo "== end $(date +%T)"
