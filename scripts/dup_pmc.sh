#!/usr/bin/env bash
# Differential instruction counts per section (VPT_DUP builds, csrc/vpt_device.h): one rocprofv3 PMC pass
# (8 SQ instruction counters) over one bench step -- FF configs[1] + the north-star MIS + HG configs[2],
# full size -- for the release library and for each build_variants/libvpt_dup<k>.so.
# usage (GPU box): bash scripts/dup_pmc.sh <tag> base dup1 dup2 ...   then: python scripts/dup_summary.py gpurun_out/dup_<tag>
set -u
TAG=${1:?tag}; shift
OUT=gpurun_out/dup_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CTRS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SMEM"
for v in "$@"; do
    lib=minimal_volumetric_path_tracer_amd/libvpt.so
    case $v in base*) ;; *) lib=build_variants/libvpt_$v.so ;; esac
    [ -f "$lib" ] || { echo "STOP: $lib missing"; exit 2; }
done
for v in "$@"; do
    lib=minimal_volumetric_path_tracer_amd/libvpt.so
    case $v in base*) ;; *) lib=build_variants/libvpt_$v.so ;; esac
    VPT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace -d "$OUT/$v" -o run --output-format csv -- \
        python3 bench.py --config ff --steps 1 --warmup 0 --no-cpu --inflight 1 > "$OUT/$v.log" 2>&1
    rc=$?
    echo "$v rc=$rc"
    case $rc in 0) ;; *) tail -5 "$OUT/$v.log"; echo "STOP"; exit $rc ;; esac
done
echo "== done"
