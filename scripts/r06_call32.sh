set -u
export TMPDIR=/tmp
REPS=2 bash scripts/ab.sh r06y base fm0b fmm || exit $?
echo "== end $(date +%T)"
