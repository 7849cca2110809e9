set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06m base fm || exit $?
echo "== end $(date +%T)"
