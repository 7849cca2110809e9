#!/usr/bin/env bash
# round 6: the EST = 1 unit with the default machine scheduler, and its stage / tracker / bias options
set -u
REPS=3 bash scripts/ab.sh r06misched2 base misdef dtrk dnuc dncl db0
