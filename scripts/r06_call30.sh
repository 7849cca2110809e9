set -u
export TMPDIR=/tmp
bash scripts/sect_run.sh r06s5 sect || exit $?
echo "== end $(date +%T)"
