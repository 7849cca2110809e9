#!/usr/bin/env bash
# PMC counter passes over one bench step (each pass its own rocprofv3 run, kernel-trace only).
# usage: bash scripts/pmc.sh <tag> [bench args...]
set -u
TAG=${1:-r01}
shift || true
ARGS=${*:---steps 1 --warmup 0 --no-cpu --inflight 1}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM"
  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_CVT"
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VSKIPPED GRBM_GUI_ACTIVE"
  "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_LEVEL_WAVES"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_WAVES"
)
# PMC_PASSES="A B;C D" replaces the list (one pass per ';'-separated group)
if [ -n "${PMC_PASSES:-}" ]; then IFS=';' read -r -a PASSES <<< "$PMC_PASSES"; fi
i=0
for p in "${PASSES[@]}"; do
    i=$((i + 1))
    echo "== pass $i: $p"
    timeout -k 10 ${PMC_TIMEOUT:-600} rocprofv3 --pmc $p --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- \
        python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "rc=$rc"
    case $rc in 0) ;; *) tail -5 "$OUT/p$i.log"; echo "STOP"; exit $rc ;; esac
done
echo "== done"
