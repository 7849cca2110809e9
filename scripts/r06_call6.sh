set -u
export TMPDIR=/tmp
REPS=3 bash scripts/ab.sh r06e base notakein noacossel norareb || exit $?
echo "== end $(date +%T)"
