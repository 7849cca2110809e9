#!/usr/bin/env bash
# Round 6, final build: wait attribution by memory class (PMC passes) and the section-timer profile
# (VPT_SECTIONS build of the same sources, build_variants/libvpt_sect.so).  Any failure ends the script.
set -u
bash scripts/wait_attrib.sh r06w || exit $?
bash scripts/sect_run.sh r06s sect || exit $?
echo "== call10 done"
