#!/usr/bin/env bash
# round 6: the point-light shadow ray cast in the light cone ray's pass for lanes whose light sphere test fails (VPT_SS_FUSE)
set -u
REPS=3 bash scripts/ab.sh r06ssf base ssfuse
