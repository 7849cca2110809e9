"""Per-section dynamic instruction counts from scripts/dup_pmc.sh: PMC of each VPT_DUP=k build (section k
run twice) minus the release build's, for pool_kernel<0> (FF configs[1]) and pool_kernel<1> (MIS + HG
configs[2]).  Counts in G wave-instructions per launch.

    python scripts/dup_summary.py gpurun_out/dup_<tag> > profiles/r06/dup_sections.txt
"""
import csv
import glob
import os
import sys

NAMES = {"dup1": "decide (whole)", "dup2": "decide: intersection", "dup3": "surface event (whole)",
         "dup4": "S: MISv2 (two lights)", "dup5": "S: MISv2 ray casts", "dup6": "medium event (whole)",
         "dup7": "M: single scattering", "dup8": "M: equi-angular setup", "dup9": "S: pLight",
         "dup10": "S: bdsf + update", "dup11": "M: phase sample", "dup12": "A: camera ray",
         "dup13": "task load + store", "dup14": "M: ss cone ray cast", "dup15": "M: ss cone direction",
         "dup16": "S: MISv2 cone trig (2 dirs)"}
CTR = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
       "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT32", "SQ_INSTS_SMEM"]


def counters(d, pattern):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None
    rows = list(csv.DictReader(open(f[0])))
    ids = [r["Dispatch_Id"] for r in rows if pattern in r["Kernel_Name"]]
    if not ids:
        return None
    did = ids[-1]
    c = {}
    for r in rows:
        if r["Dispatch_Id"] == did:
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return c


def derived(c):
    fp64 = sum(c[k] for k in CTR[2:6])
    return {"valu": c["SQ_INSTS_VALU"], "fp64": fp64, "nonfp64": c["SQ_INSTS_VALU"] - fp64,
            "int32": c["SQ_INSTS_VALU_INT32"], "trans": c["SQ_INSTS_VALU_TRANS_F64"], "salu": c["SQ_INSTS_SALU"],
            "smem": c["SQ_INSTS_SMEM"]}


def main():
    root = sys.argv[1]
    vs = sorted((os.path.basename(p) for p in glob.glob(os.path.join(root, "*")) if os.path.isdir(p)),
                key=lambda v: (not v.startswith("base"), int(v[3:]) if v[3:].isdigit() else 0, v))
    for est, pat in (("FF configs[1] 1024^2 x 256", "pool_kernel<0"), ("MIS + HG configs[2] 1024^2 x 1024", "pool_kernel<1")):
        base = [derived(c) for v in vs if v.startswith("base") for c in [counters(os.path.join(root, v), pat)] if c]
        if not base:
            continue
        b = {k: sum(x[k] for x in base) / len(base) for k in base[0]}
        print(f"# {est}: release build, G wave-instructions per launch (mean of {len(base)} runs)")
        print(f"{'':30s} {'VALU':>8s} {'FP64':>8s} {'nonFP64':>8s} {'INT32':>8s} {'TRANS':>7s} {'SALU':>8s} {'SMEM':>7s}")
        row = lambda name, x: print(f"{name:30s} {x['valu']/1e9:8.3f} {x['fp64']/1e9:8.3f} {x['nonfp64']/1e9:8.3f} "
                                    f"{x['int32']/1e9:8.3f} {x['trans']/1e9:7.3f} {x['salu']/1e9:8.3f} {x['smem']/1e9:7.3f}")
        row("total", b)
        if len(base) > 1:
            sp = {k: (max(x[k] for x in base) - min(x[k] for x in base)) for k in b}
            row("  run-to-run spread", sp)
        print("# sections: counts of the VPT_DUP=k build minus the release build's")
        for v in vs:
            if v.startswith("base"):
                continue
            c = counters(os.path.join(root, v), pat)
            if not c:
                continue
            d = derived(c)
            row(f"{NAMES.get(v, v)}", {k: d[k] - b[k] for k in b})
        print()


if __name__ == "__main__":
    main()
