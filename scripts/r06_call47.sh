#!/usr/bin/env bash
# Round 6, final build 434066a7: wait attribution by memory class (PMC passes) and the section-timer profile
# (VPT_SECTIONS build of the same sources, build_variants/libvpt_sect.so).  Any failure ends the script.
set -u
bash scripts/wait_attrib.sh r06w6 || exit $?
bash scripts/sect_run.sh r06s6 sect || exit $?
echo "== call47 done"
