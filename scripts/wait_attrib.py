"""Which memory class the pool kernel's waves wait on (Missing #3): summarises the passes of
scripts/wait_attrib.sh (rocprofv3 --pmc, one counter group per class) into profiles/<round>/wait_attrib_*.json.

    python scripts/wait_attrib.py gpurun_out/pmc_<tag> 'pool_kernel<1, false>' > profiles/r05/wait_attrib_mis.json

Per class (VMEM = global / scratch loads and stores, SMEM = scalar loads, LDS, instruction fetch) the
profiler's derived latency metric is the class's summed in-flight level (SQ_INST_LEVEL_* accumulated
every cycle) over its instruction count, i.e. the mean cycles from issue to data.  Latency x count is
the class's in-flight instruction-cycles; over SQ_WAVE_CYCLES (the wave-cycles of the dispatch) it is
the number of such instructions the average wave has outstanding -- an upper bound on the share of
wave-time that waits on the class (instructions of one wave in flight together count once each; a
wave that waits on two classes at once counts in both).  SQ_WAIT_ANY / SQ_WAVE_CYCLES is the share
actually spent parked in s_waitcnt, for scale."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import build_id_of, last_dispatch  # noqa: E402

CLASSES = {
    # class: (latency metric, instruction counter); SQ_INSTS_VMEM = VMEM_RD + VMEM_WR when not collected
    "vmem": ("VmemLatency", "SQ_INSTS_VMEM"),
    "smem": ("SmemLatency", "SQ_INSTS_SMEM_NORM"),
    "lds": ("LdsLatency", "SQ_INSTS_LDS"),
    "ifetch": ("InstrFetchLatency", "SQ_IFETCH"),
}


def main():
    """argv: <pmc dir> <kernel pattern> [<pmc_summary JSON of the same build>: instruction counts the
    passes did not collect, e.g. profiles/r04/pmc_pool_kernel_mis.json]"""
    d, pat = sys.argv[1], sys.argv[2]
    dispatch, c = None, {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        info, cc = last_dispatch(f, pat)
        if info:
            dispatch = dispatch or info
            for k, v in cc.items():  # SQ_WAVE_CYCLES etc. appear in several passes: keep the first
                c.setdefault(k, v)
    if not dispatch:
        raise SystemExit(f"no dispatch matching {pat!r} under {d}")
    if "SQ_INSTS_VMEM" not in c and "SQ_INSTS_VMEM_RD" in c:
        c["SQ_INSTS_VMEM"] = c["SQ_INSTS_VMEM_RD"] + c.get("SQ_INSTS_VMEM_WR", 0)
    filled = {}
    if len(sys.argv) > 3:
        ref = json.load(open(sys.argv[3]))
        for name, (lat, cnt) in CLASSES.items():
            alt = "SQ_INSTS_SMEM" if cnt == "SQ_INSTS_SMEM_NORM" else cnt
            if cnt not in c and alt in ref["counters"]:
                c[cnt] = ref["counters"][alt]
                filled[cnt] = f"{alt} from {sys.argv[3]} (build {ref.get('build_id')})"
    # SQ_WAVE_CYCLES counts quad-cycles (x4 = the dispatch's wave-cycles: 2048 waves x its 448 M
    # cycles per XCD for MIS + HG); the latency metrics are in cycles (LDS 75, instruction fetch 17)
    wc = 4 * c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None
    out = {"source": f"rocprofv3 --pmc, one pass per class (scripts/wait_attrib.sh), {os.path.basename(d)}",
           "build_id": build_id_of(d), "dispatch": dispatch, "counters": c, "filled_from_profile": filled,
           "units": "latency_cycles: cycles from issue to data; per_wave_cycle: in-flight instructions of the class "
                    "per wave-cycle (latency x count / (4 x SQ_WAVE_CYCLES)); *_per_wave_cycle under derived: "
                    "counter / wave-cycles",
           "classes": {}}
    for name, (lat, cnt) in CLASSES.items():
        L, N = c.get(lat), c.get(cnt)
        rec = {"latency_cycles": L, "instructions": N}
        if L is not None and N:
            rec["inflight_inst_cycles"] = L * N
            if wc:
                rec["per_wave_cycle"] = L * N / wc
        out["classes"][name] = rec
    der = {}
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_LDS"):  # quad-cycle counters, as SQ_WAVE_CYCLES
            if c.get(k) is not None:
                der[k.lower() + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
    if c.get("SQC_DCACHE_REQ"):
        der["sqc_dcache_miss_rate"] = (c.get("SQC_DCACHE_MISSES") or 0) / c["SQC_DCACHE_REQ"]
    if c.get("SQC_ICACHE_HITS") is not None and c.get("SQC_ICACHE_MISSES") is not None:
        der["sqc_icache_miss_rate"] = c["SQC_ICACHE_MISSES"] / max(1.0, c["SQC_ICACHE_HITS"] + c["SQC_ICACHE_MISSES"])
    if c.get("TCP_TCC_READ_REQ_sum"):
        der["l1_to_l2_read_latency_cycles"] = c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / c["TCP_TCC_READ_REQ_sum"]
    if c.get("SQ_INSTS_VMEM") and c.get("SQ_INSTS_FLAT") is not None:
        der["flat_share_of_vmem"] = c["SQ_INSTS_FLAT"] / c["SQ_INSTS_VMEM"]
    # instruction fetch overlaps issue (prefetch); s_waitcnt waits on VMEM (vmcnt) or SMEM + LDS (lgkmcnt)
    ranked = sorted(((v.get("per_wave_cycle") or 0, k) for k, v in out["classes"].items() if k != "ifetch"),
                    reverse=True)
    der["dominant_class"] = ranked[0][1] if ranked and ranked[0][0] > 0 else None
    out["derived"] = der
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
