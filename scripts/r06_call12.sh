set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06i base fc1 g1 g3 g1np || exit $?
echo "== end $(date +%T)"
