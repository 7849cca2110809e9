#!/usr/bin/env bash
# round 6: machine-scheduler strategies for the EST = 1 unit only (vpt_pool_mis.hip), the main unit unchanged
set -u
REPS=3 bash scripts/ab.sh r06misched base misdef misilp mismc mismr
