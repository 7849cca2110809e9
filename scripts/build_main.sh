#!/usr/bin/env bash
# The in-tree libvpt.so build under the lock scripts/build_variant.sh takes, so variant builds can run beside it.
exec flock /tmp/vpt_build_variant.lock make -s -C "$(dirname "$0")/../minimal_volumetric_path_tracer_amd/csrc" "$@"
