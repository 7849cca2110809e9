#!/usr/bin/env bash
# round 6: deferred point-light shadow rays of medium events in a ring of their own (VPT_MED_DEFER)
set -u
REPS=3 bash scripts/ab.sh r06def base defer
