"""Per-section opcode-class budget of pool_kernel<EST> from its code object.

Each instruction of the kernel (and of the out-of-line libm entry points it calls) is classed by opcode
(FP64 arithmetic, v_cndmask, v_mov, v_cmp, other VALU / integer, readlane/writelane, SALU, branch,
SMEM, VMEM, LDS, s_nop, s_waitcnt) and attributed to a section of the section-timer profile
(csrc/vpt_device.h SECT_*) by its inline stack (llvm-symbolizer --inlines on a build with line tables:
`-gline-tables-only` changes the schedule slightly, not the instruction mix).  The static counts of a
section's straight-line code times the section's entries per launch (a sections_*.txt profile) give
the dynamic budget; rare branches inside a section (libm rare arguments, the metal ring) make the
static count an upper bound there.

usage: python scripts/isa_mix.py <code object .co> <est 0|1> [sections.txt] > profiles/r04/isa_mix_<est>.txt
(the .co: hipcc --cuda-device-only -c -gline-tables-only ... vpt_kernels.hip -- for est 1, vpt_pool_mis.hip with
 the Makefile's MISFLAGS, the unit that holds that kernel -- then
 clang-offload-bundler --unbundle --targets=hipv4-amdgcn-amd-amdhsa--gfx950)"""
import collections
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin/"
CLASSES = ["fp64", "cndmask", "mov", "cmp", "valu_int", "lane", "salu", "branch", "smem", "vmem", "lds", "nop", "waitcnt"]


def op_class(op):
    if op.startswith("v_"):
        if op.startswith("v_cndmask"):
            return "cndmask"
        if op.startswith("v_mov") or op.startswith("v_pk_mov"):
            return "mov"
        if op.startswith("v_cmp"):
            return "cmp"
        if op.startswith("v_readlane") or op.startswith("v_writelane") or op.startswith("v_readfirstlane"):
            return "lane"
        if "_f64" in op:
            return "fp64"
        return "valu_int"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc", "s_getpc")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "salu"


# innermost-first: the first frame name that matches decides the section
RULES = [
    ("point_shadow_ld", "M shadow (in)"),
    ("phase_sample", "M phase"),
    ("eqa_medium", "M eqa"),
    ("scene_intersect_n", "S MISv2 isect3"),
    ("mis_v2", "S MISv2"),
    ("p_light", "S pLight"),
    ("bdsf", "S bdsf+update"),
    ("solid_angle_dir", "@cone"),
    ("single_scattering", "M single_scat"),
    ("medium_tail", "M tail"),
    ("medium_event", "M other"),
    ("medium_shadow_event", "M shadow (in)"),
    ("surface_event", "S other"),
    ("continue_path", "roulette"),
    ("scene_intersect_grouped", "@isect"),
    ("decide", "A decide"),
    ("pool_camera_dir", "A camera (in)"),
    ("decode_unit", "A unit handout"),
    ("store_partial", "A prep"),
    ("stage_a", "A prep"),
    ("load_task", "load_task"),
    ("store_task", "store_task"),
    ("run_event", "run_event (merged)"),
    ("pool_kernel", "sched"),
]


def section(frames):
    sec = None
    for f in frames:  # innermost first
        for key, name in RULES:
            if key in f:
                if name == "@cone":
                    return "M ss cone dir" if any("single_scattering" in g for g in frames) else "S cone/cos"
                if name == "@isect":
                    if any("decide" in g for g in frames):
                        return "A decide isect"
                    if any("single_scattering" in g for g in frames):
                        return "M ss cone isect"
                    if any("p_light" in g for g in frames):
                        return "S pLight"
                    return "isect other"
                return name
    return sec or "other"


def main():
    co, est = sys.argv[1], int(sys.argv[2])
    sect_entries = {}
    if len(sys.argv) > 3:
        for line in open(sys.argv[3]):
            m = re.match(r"\s+(.+?)\s+share\s+[\d.]+\s+entries\s+(\d+)", line)
            if m:
                sect_entries[m.group(1).strip()] = int(m.group(2))
    dis = subprocess.run([LLVM + "llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True, text=True).stdout
    kern = f"_ZN3vpt11pool_kernelILi{est}ELb0EE"
    funcs, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            cur = m.group(2)
            funcs[cur] = []
            continue
        m = re.match(r"^\s+(\S+)\s.*//\s*([0-9A-F]+):", line) or re.match(r"^\s+(\S+)\s*//\s*([0-9A-F]+):", line)
        if m and cur:
            funcs[cur].append((int(m.group(2), 16), m.group(1)))
    kname = [f for f in funcs if f.startswith(kern)][0]
    # the kernel plus the out-of-line libm entry points (gm_*) and fr_microfacet it calls
    names = [kname] + sorted(f for f in funcs if re.search(r"gm_sincos|fr_microfacet|gl_", f))
    insts = [(a, op, f) for f in names for a, op in funcs[f]]
    addrs = "\n".join(hex(a) for a, _, _ in insts)
    sym = subprocess.run([LLVM + "llvm-symbolizer", "--obj=" + co, "--inlines", "--functions=short"], input=addrs,
                         capture_output=True, text=True).stdout
    blocks = [b for b in sym.split("\n\n")]
    table = collections.defaultdict(collections.Counter)
    rare = 0
    for (a, op, f), blk in zip(insts, blocks):
        frames = [l for i, l in enumerate(blk.strip().splitlines()) if i % 2 == 0]
        # the rare rings' code (metal / other materials: surface_event<.., MK = 1 or -1>; the sequential
        # MISv2, which the diffuse rings compile but do not run with two MIS lights) is left out: the
        # budget is of what the hot rings execute.  So are the translated glibc functions (gl_*) that the
        # gm_* restatements call behind GM_UNLIKELY for rare arguments (atan2 with x <= 0, tan beyond 25).
        # Instructions whose innermost line is run_event itself are code the compiler merged across the
        # ring branches (their inlined frames are lost): "run_event (merged)", no entry count.
        if any(re.search(r"surface_event<\d+, false, (1|-1),", g) for g in frames) or \
                any(g.startswith("mis_v2<") for g in frames) or any(g.startswith("gl_") for g in frames):
            rare += 1
            continue
        sec = section(frames) if f == kname else "call " + re.sub(r"^_ZL?\d+", "", f)[:28]
        table[sec][op_class(op)] += 1
    hdr = f"{'section':22s} {'total':>6s} " + " ".join(f"{c:>8s}" for c in CLASSES) + "  non-fp64 VALU"
    print(f"# static opcode classes of {kname} ({co}); 'x entries' = static x section entries per launch")
    print(f"# ({rare} instructions of the rare rings -- metal / other materials, sequential MISv2 -- and of the")
    print("#  translated glibc fallbacks gl_* for rare arguments left out)")
    print(hdr)
    tot = collections.Counter()
    for sec in sorted(table, key=lambda s: -sum(table[s].values())):
        c = table[sec]
        tot.update(c)
        n = sum(c.values())
        nf = c["cndmask"] + c["mov"] + c["cmp"] + c["valu_int"] + c["lane"]
        print(f"{sec:22s} {n:6d} " + " ".join(f"{c[k]:8d}" for k in CLASSES) + f"  {nf:6d}")
    n = sum(tot.values())
    print(f"{'TOTAL':22s} {n:6d} " + " ".join(f"{tot[k]:8d}" for k in CLASSES))
    if sect_entries:
        print("\n# weighted by entries (millions of wave-instructions per launch, straight-line estimate)")
        print(f"{'section':22s} {'entries':>10s} {'all':>8s} {'fp64':>8s} {'sel/mov/cmp':>12s} {'int/lane':>9s} {'salu+br':>8s}")
        for sec in sorted(table, key=lambda s: -sum(table[s].values()) * sect_entries.get(s, 0)):
            e = sect_entries.get(sec)
            if not e:
                continue
            c = table[sec]
            w = lambda k: c[k] * e / 1e6
            print(f"{sec:22s} {e:10d} {sum(c.values()) * e / 1e6:8.1f} {w('fp64'):8.1f} "
                  f"{(c['cndmask'] + c['mov'] + c['cmp']) * e / 1e6:12.1f} {(c['valu_int'] + c['lane']) * e / 1e6:9.1f} "
                  f"{(c['salu'] + c['branch']) * e / 1e6:8.1f}")


if __name__ == "__main__":
    main()
