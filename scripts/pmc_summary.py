"""Summarise the rocprofv3 PMC passes of scripts/pmc.sh into one JSON (profiles/<round>/pmc_*.json).

    python scripts/pmc_summary.py gpurun_out/pmc_r01 'pool_kernel<0, false>' > profiles/r01/pmc_pool_kernel.json

Records the build id the passes ran (from bench.py's JSON line in each pass's log); bench.py uses the
profile only for the library with that id.

Takes, in every pass, the LAST dispatch whose kernel name contains the pattern (bench.py runs the
counting build first, then the timed launch), and derives lane utilisation, wait fractions and HBM
bytes.  gfx950: FETCH_SIZE counts half of a streamed read, so HBM reads = 2 * FETCH_SIZE KiB
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section); WRITE_SIZE is in KiB as reported.
"""
import csv
import glob
import json
import os
import sys


def last_dispatch(path, pattern):
    rows = list(csv.DictReader(open(path)))
    ids = [r["Dispatch_Id"] for r in rows if pattern in r["Kernel_Name"]]
    if not ids:
        return None, {}
    did = ids[-1]
    sel = [r for r in rows if r["Dispatch_Id"] == did]
    counters = {}
    for r in sel:
        counters[r["Counter_Name"]] = counters.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    r0 = sel[0]
    info = {"kernel": r0["Kernel_Name"], "grid": r0["Grid_Size"], "workgroup": r0["Workgroup_Size"],
            "lds_bytes": r0["LDS_Block_Size"], "scratch": r0["Scratch_Size"], "vgpr": r0["VGPR_Count"],
            "agpr": r0["Accum_VGPR_Count"], "sgpr": r0["SGPR_Count"],
            "duration_ns": int(r0["End_Timestamp"]) - int(r0["Start_Timestamp"])}
    return info, counters


def build_id_of(d):
    """the library build every pass ran (bench.py's JSON line prints vpt.build_id()); the passes must agree,
    so bench.py can tie the counters to the library it loads"""
    ids = set()
    for f in sorted(glob.glob(os.path.join(d, "p*.log"))):
        for line in open(f):
            if line.startswith("{"):
                try:
                    ids.add(json.loads(line).get("build_id"))
                except ValueError:
                    pass
    if len(ids) != 1 or None in ids:
        raise SystemExit(f"passes under {d} ran builds {sorted(map(str, ids))}: expected exactly one")
    return ids.pop()


def main():
    d, pat = sys.argv[1], sys.argv[2]
    dispatch, c = None, {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        info, cc = last_dispatch(f, pat)
        if info:
            dispatch = dispatch or info
            c.update(cc)
    if not dispatch:
        raise SystemExit(f"no dispatch matching {pat!r} under {d}")
    g = lambda k: c.get(k)
    der = {}
    if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
        der["valu_lane_utilization"] = g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU"))
    if g("SQ_WAVE_CYCLES"):
        wc = g("SQ_WAVE_CYCLES")
        if g("SQ_ACTIVE_INST_ANY"):
            der["wave_cycles_issuing_frac"] = g("SQ_ACTIVE_INST_ANY") / wc
        # MI355X_MICROARCH.md: SQ_WAIT_ANY = wave parked (s_waitcnt / barrier / sleep), SQ_WAIT_INST_ANY =
        # issue stall (dependency / pipe); with ACTIVE_INST_ANY they partition WAVE_CYCLES
        if g("SQ_WAIT_ANY"):
            der["wave_cycles_waitcnt_frac"] = g("SQ_WAIT_ANY") / wc
        if g("SQ_WAIT_INST_ANY"):
            der["wave_cycles_issue_stall_frac"] = g("SQ_WAIT_INST_ANY") / wc
        if g("SQ_WAIT_INST_LDS"):
            der["wave_cycles_wait_lds_frac"] = g("SQ_WAIT_INST_LDS") / wc
    if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
        der["valu_insts_per_wave"] = g("SQ_INSTS_VALU") / g("SQ_WAVES")
    f64 = sum(g(k) or 0 for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                  "SQ_INSTS_VALU_TRANS_F64"))
    if f64:
        der["fp64_valu_insts"] = f64
        if g("SQ_INSTS_VALU"):
            der["fp64_share_of_valu"] = f64 / g("SQ_INSTS_VALU")
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_LDS_IDX_ACTIVE"):
        der["lds_bank_conflict_frac"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
    if g("FETCH_SIZE") is not None:
        der["hbm_read_bytes_fetch_size_x2"] = 2 * g("FETCH_SIZE") * 1024
    if g("WRITE_SIZE") is not None:
        der["hbm_write_bytes"] = g("WRITE_SIZE") * 1024
    if g("GRBM_GUI_ACTIVE"):
        der["effective_clock_ghz"] = g("GRBM_GUI_ACTIVE") / 8 / dispatch["duration_ns"]  # summed over 8 XCDs
        if g("SQ_ACTIVE_INST_VALU"):  # quad-cycles of VALU issue summed over waves, per SIMD-cycle (1024 SIMDs)
            der["simd_valu_busy_frac"] = 4 * g("SQ_ACTIVE_INST_VALU") / (1024 * g("GRBM_GUI_ACTIVE") / 8)
    if g("SQ_LEVEL_WAVES") and g("SQ_BUSY_CYCLES"):
        der["mean_resident_waves_per_se"] = g("SQ_LEVEL_WAVES") / g("SQ_BUSY_CYCLES")
    out = {"source": f"rocprofv3 --pmc <counters> --kernel-trace, one pass per counter group (scripts/pmc.sh), "
                     f"{os.path.basename(d)}", "build_id": build_id_of(d), "dispatch": dispatch, "counters": c,
           "derived": der}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
