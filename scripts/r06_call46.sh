#!/usr/bin/env bash
# round 6 final measurement of build 434066a7 (VPT_SS_FUSE)
set -u
bash scripts/final_run.sh r06final6 r06
