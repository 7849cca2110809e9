#!/usr/bin/env bash
# round 6: the sphere tests' rare-argument test read from the square-root core's first product (VPT_ISECT_NAN)
set -u
REPS=3 bash scripts/ab.sh r06nan base isnan
