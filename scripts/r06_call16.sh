set -u
export TMPDIR=/tmp
REPS=3 bash scripts/ab.sh r06l base vidx || exit $?
echo "== end $(date +%T)"
