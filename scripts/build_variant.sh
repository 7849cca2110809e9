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
flock /tmp/vpt_build_variant.lock make -s -C "$C" vpt_host.o vpt_multi.o  # (the in-tree make takes the same lock: scripts/build_main.sh)
# the Makefile's flags (SCHED: the scheduler strategy; SCHED= builds with the compiler's default; OPT: -O level)
SCHED=${SCHED--mllvm -amdgpu-sched-strategy=iterative-maxocc}
LOOPFLAGS=${LOOPFLAGS--mllvm -disable-lsr}
FLAGS="--offload-arch=${VARCH:-gfx950} ${OPT:--O2} -std=c++17 -fPIC -ffp-contract=off -fno-fast-math $SCHED $LOOPFLAGS -Wno-unused-function $*"
MISFLAGS=${MISFLAGS--mllvm -disable-machine-licm}  # the EST = 1 pool kernel's unit (csrc/Makefile MISFLAGS)
MAINFLAGS=${MAINFLAGS-}  # extra flags for vpt_kernels.hip only (every kernel but the EST = 1 pool kernel)
/opt/rocm/bin/hipcc $FLAGS $MAINFLAGS -c "$C/vpt_kernels.hip" -o "build_variants/vpt_kernels_$name.o"
/opt/rocm/bin/hipcc $FLAGS $MISFLAGS -c "$C/vpt_pool_mis.hip" -o "build_variants/vpt_pool_mis_$name.o"
# the variant's own build id (sources + its flags + its name), so a result measured on a variant is
# never recorded under the production library's id
VID=$(python3 scripts/build_id.py "variant:$name | $FLAGS | $MAINFLAGS | $MISFLAGS")
echo "const char* vpt_build_id(void) { return \"$VID\"; }" > "build_variants/vpt_build_id_$name.c"
cc -O2 -fPIC -c "build_variants/vpt_build_id_$name.c" -o "build_variants/vpt_build_id_$name.o"
/opt/rocm/bin/hipcc --offload-arch=${VARCH:-gfx950} -shared -fPIC "build_variants/vpt_kernels_$name.o" "build_variants/vpt_pool_mis_$name.o" "$C/vpt_host.o" "$C/vpt_multi.o" "build_variants/vpt_build_id_$name.o" \
    -o "build_variants/libvpt_$name.so" -lpthread -L/opt/rocm/lib -lrccl
echo "build_variants/libvpt_$name.so"
