#!/usr/bin/env bash
# round 6 closing check on the shipped tree: GPU parity tests, smoke, default bench
set -u
bash scripts/gpu_check.sh r06close tests smoke bench
