set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06q base lsr0 ssm || exit $?
echo "== end $(date +%T)"
