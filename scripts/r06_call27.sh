set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06v base ng10 ng2 dg10 prio0 || exit $?
echo "== end $(date +%T)"
