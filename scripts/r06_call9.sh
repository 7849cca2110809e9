set -u
export TMPDIR=/tmp
REPS=3 bash scripts/ab.sh r06g base db hgsel || exit $?
echo "== end $(date +%T)"
