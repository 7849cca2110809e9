set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06u base mcse0 prera0 ovl0 eli || exit $?
echo "== end $(date +%T)"
