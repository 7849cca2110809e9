#!/usr/bin/env bash
# CPU-only compile study of a split (one kernel per pool stage) design: VGPR / SGPR / spills of each stage
# kernel of scripts/split_study.hip at 2, 3 and 4 waves per SIMD, product flags.  No GPU.
# usage: [EXTRA=flags] bash scripts/split_study.sh [est] > profiles/r06/split_resources.txt (estimator 1: EXTRA="-mllvm -disable-machine-licm", its unit's flags)
set -eu
cd "$(dirname "$0")/.."
EST=${1:-1}
C=minimal_volumetric_path_tracer_amd/csrc
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
FLAGS="--offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off -fno-fast-math -mllvm -amdgpu-sched-strategy=iterative-maxocc -mllvm -disable-lsr ${EXTRA:-}"
echo "# split-kernel compile study, estimator $EST (hipcc $FLAGS); per stage kernel and waves/SIMD target W:"
echo "# vgpr (budget 512/W), sgpr, spilled VGPRs / SGPRs, scratch bytes per lane, static instructions of the kernel body"
printf "%-10s %2s %5s %5s %6s %6s %8s %7s\n" kernel W vgpr sgpr vspill sspill scratch insts
for W in 2 3 4; do
    /opt/rocm/bin/hipcc $FLAGS --cuda-device-only -S -I$C -DSPLIT_W=$W -DSPLIT_EST=$EST scripts/split_study.hip \
        -o "$TMP/s$W.s" 2>/dev/null
    python3 - "$TMP/s$W.s" "$W" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
W = sys.argv[2]
maps = re.split(r"\n  - ", txt[txt.index("amdhsa.kernels:"):])
for k in ("k_decide", "k_surf_d", "k_med", "k_surf_r"):
    rec = [mp for mp in maps if re.search(r"\.name:\s+_Z\d+" + k + r"\d", mp)][0]
    get = lambda f: int(re.search(r"\." + f + r":\s+(\d+)", rec).group(1))
    sym = re.search(r"\.name:\s+(\S+)", rec).group(1)
    body = txt[txt.index("\n" + sym + ":"):]
    body = body[:body.index(".Lfunc_end")]
    ninst = sum(1 for l in body.splitlines() if l.startswith("\t") and not l.startswith("\t.") and l.strip()
                and not l.strip().startswith(";"))
    print(f"{k:10s} {W:>2s} {get('vgpr_count'):5d} {get('sgpr_count'):5d} {get('vgpr_spill_count'):6d} "
          f"{get('sgpr_spill_count'):6d} {get('private_segment_fixed_size'):8d} {ninst:7d}")
PY
done
