set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06w base fo3 fmb0 fas0 || exit $?
echo "== end $(date +%T)"
