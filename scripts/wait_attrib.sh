#!/usr/bin/env bash
# PMC passes that split the pool kernel's s_waitcnt time by memory class (Missing #3):
# one rocprofv3 run per class, each within the per-block counter limits (<= 8 SQ/SQC, <= 4 TCP).
# One bench step measures FF (configs[1]) then MIS + HG (configs[2]); scripts/wait_attrib.py summarises
# each kernel.
# usage: bash scripts/wait_attrib.sh <tag>   (on the GPU box; writes gpurun_out/pmc_<tag>/)
set -u
TAG=${1:?tag}
export PMC_TIMEOUT=${PMC_TIMEOUT:-240}
export PMC_PASSES="VmemLatency SQ_INSTS_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAVE_CYCLES SQ_WAIT_ANY;\
SmemLatency SQ_INSTS_SMEM_NORM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VMEM_RD;\
LdsLatency SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS;\
InstrFetchLatency SQ_IFETCH SQ_WAVE_CYCLES SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_BUSY_CYCLES;\
SQC_DCACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_REQ SQ_WAVE_CYCLES TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
bash scripts/pmc.sh "$TAG" --steps 1 --warmup 0 --no-cpu --inflight 1 || exit $?
mkdir -p gpurun_out/wait_$TAG
python3 scripts/wait_attrib.py "gpurun_out/pmc_$TAG" 'pool_kernel<0, false>' > "gpurun_out/wait_$TAG/wait_attrib_ff.json" || exit 1
python3 scripts/wait_attrib.py "gpurun_out/pmc_$TAG" 'pool_kernel<1, false>' > "gpurun_out/wait_$TAG/wait_attrib_mis.json" || exit 1
python3 - "$TAG" <<'EOF'
import json, sys
for k in ("ff", "mis"):
    d = json.load(open(f"gpurun_out/wait_{sys.argv[1]}/wait_attrib_{k}.json"))
    print(k, {c: round(v.get("per_wave_cycle") or 0, 4) for c, v in d["classes"].items()},
          {c: round(v.get("latency_cycles") or 0, 1) for c, v in d["classes"].items()}, d["derived"])
EOF
