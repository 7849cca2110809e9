set -u
export TMPDIR=/tmp
REPS=3 bash scripts/ab.sh r06d base noframe rareb || exit $?
echo "== end $(date +%T)"
