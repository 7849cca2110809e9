#!/usr/bin/env bash
# Round 6, final build (10ab2d20162cb9b6): wait attribution, section timers (VPT_SECTIONS build) and the
# VPT_DUP differential PMC of every section.  Any failure ends the script.
set -u
bash scripts/wait_attrib.sh r06w2 || exit $?
bash scripts/sect_run.sh r06s2 sect || exit $?
bash scripts/dup_pmc.sh r06c base dup1 dup2 dup3 dup4 dup5 dup6 dup7 dup8 dup9 dup10 dup11 dup12 dup13 dup14 dup15 dup16 || exit $?
python3 scripts/dup_summary.py gpurun_out/dup_r06c > gpurun_out/dup_r06c/summary.txt || exit 1
echo "== call14 done"
