set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06s base mlicm0 sinkav msink0 etd0 || exit $?
echo "== end $(date +%T)"
