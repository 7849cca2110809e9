#!/usr/bin/env bash
# PMC of the pool kernel for libvpt.so variants (build_variants/libvpt_<name>.so; "base" = in-tree):
# two short passes each (one FF bench step; PMCV_ARGS= also runs the north-star MIS + HG step, for
# PMC_KERNEL="pool_kernel<1, false>"), summarised per variant.  usage: bash scripts/pmc_var.sh name...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
P1=${P1:-"SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS"}
P2=${P2:-"TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_EA0_WRREQ_sum"}
# the timed dispatch only (bench.py runs the counting build, pool_kernel<EST, true>, first)
export PMC_KERNEL=${PMC_KERNEL:-"pool_kernel<0, false>"}
for v in "$@"; do
    lib=build_variants/libvpt_$v.so
    [ "$v" = base ] && lib=minimal_volumetric_path_tracer_amd/libvpt.so
    i=0
    for p in "$P1" "$P2"; do
        i=$((i + 1))
        VPT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace -d gpurun_out/pmcv_$v/p$i -o run --output-format csv -- \
            python3 bench.py --steps 1 --warmup 0 --no-cpu --inflight 1 ${PMCV_ARGS---no-north-star} > gpurun_out/pmcv_${v}_p$i.log 2>&1
        rc=$?
        if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcv_${v}_p$i.log; echo "STOP rc=$rc"; exit $rc; fi
    done
    python3 - "$v" <<'PY'
import csv, glob, os, sys, collections
v = sys.argv[1]
acc, dur = collections.defaultdict(float), []
for p in glob.glob(f"gpurun_out/pmcv_{v}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if os.environ["PMC_KERNEL"] in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
for p in glob.glob(f"gpurun_out/pmcv_{v}/p1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if os.environ["PMC_KERNEL"] in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(f"{v}: pool_kernel ms {dur}  " + "  ".join(f"{k} {acc[k]:.4g}" for k in sorted(acc)))
print(f"   waitany/wave_cycles {acc['SQ_WAIT_ANY'] / max(1, acc['SQ_WAVE_CYCLES']):.3f}")
PY
done
