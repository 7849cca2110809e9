#!/usr/bin/env bash
# Build an A/B variant of libvpt.so with extra compile flags into build_variants/libvpt_<name>.so
# (select it at run time with VPT_LIB=build_variants/libvpt_<name>.so, e.g. via scripts/ab.sh).
# usage: bash scripts/build_variant.sh <name> [extra hipcc flags...]
set -eu
cd "$(dirname "$0")/.."
name=$1
shift
mkdir -p build_variants
C=minimal_volumetric_path_tracer_amd/csrc
flock /tmp/vpt_build_variant.lock make -s -C "$C" vpt_host.o vpt_multi.o vpt_build_id.o
/opt/rocm/bin/hipcc --offload-arch=${VARCH:-gfx950} -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
    -Wno-unused-function "$@" -c "$C/vpt_kernels.hip" -o "build_variants/vpt_kernels_$name.o"
/opt/rocm/bin/hipcc --offload-arch=${VARCH:-gfx950} -shared -fPIC "build_variants/vpt_kernels_$name.o" "$C/vpt_host.o" "$C/vpt_multi.o" "$C/vpt_build_id.o" \
    -o "build_variants/libvpt_$name.so" -lpthread -L/opt/rocm/lib -lrccl
echo "build_variants/libvpt_$name.so"
