set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06x base eifcvt wprio nolal aa0 || exit $?
echo "== end $(date +%T)"
