"""Register / scratch / LDS budget of every kernel in libvpt.so, read from the shipped code object's
AMDGPU metadata notes (not from the profiler's dispatch record, whose VGPR_Count field is the kernel
descriptor's granulated count in 4-register units: 256 registers read as "128" there).

    python scripts/co_resources.py [minimal_volumetric_path_tracer_amd/libvpt.so] > profiles/r05/resources.txt

Steps: the .hip_fatbin section of the .so -> clang-offload-bundler (gfx950 bundle) -> llvm-readelf --notes.
gfx950 has a unified 512-entry register file per SIMD lane: a wave's arch VGPRs + AGPRs share it, so
256 registers per wave = 2 waves per SIMD (one 512-thread workgroup per CU, which the 160 KB LDS pool
fixes anyway)."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def notes(so: str) -> str:
    """the notes of every gfx950 code object in the .so: one offload bundle per HIP translation unit
    (vpt_kernels.hip, vpt_pool_mis.hip), concatenated in .hip_fatbin"""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so, os.path.join(td, "junk")],
                       check=True)
        blob = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)] + [len(blob)]
        out = []
        for k in range(len(starts) - 1):
            part, co = os.path.join(td, f"b{k}.bin"), os.path.join(td, f"k{k}.co")
            open(part, "wb").write(blob[starts[k]:starts[k + 1]])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                           check=True)
            out.append(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                      text=True).stdout)
        return "\n".join(out)


def kernels(txt: str):
    keys = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
            "private_segment_fixed_size", "group_segment_fixed_size", "max_flat_workgroup_size")
    for blk in txt.split("  - .agpr_count")[1:]:
        blk = ".agpr_count" + blk
        rec = {"name": re.search(r"\.name:\s+(\S+)", blk).group(1)}
        for k in keys:
            m = re.search(r"\." + k + r":\s+(\S+)", blk)
            rec[k] = int(m.group(1)) if m else None
        yield rec


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "minimal_volumetric_path_tracer_amd", "libvpt.so")
    sys.path.insert(0, ROOT)
    recs = sorted(kernels(notes(so)), key=lambda r: r["name"])
    def strip_args(n):  # "void vpt::k<(int)0, false>(args...)" -> "vpt::k<(int)0, false>"
        n, depth = re.sub(r"^void ", "", n).replace("(anonymous namespace)::", ""), 0
        for i, ch in enumerate(n):
            depth += ch == "<"
            depth -= ch == ">"
            if ch == "(" and depth == 0:
                return n[:i]
        return n

    short = [strip_args(n) for n in demangle([r["name"] for r in recs])]
    try:
        from minimal_volumetric_path_tracer_amd._lib import build_id
        bid = build_id()
    except Exception as e:  # noqa: BLE001 (the table is still useful without the id)
        bid = f"unknown ({e})"
    print(f"# {os.path.relpath(so, ROOT)}  build_id {bid}")
    print(f"# {'kernel':58s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'v_spill':>8s} {'s_spill':>8s} "
          f"{'scratch_B':>9s} {'lds_B':>7s} {'wg_max':>6s} {'waves/SIMD':>10s}")
    for r, n in zip(recs, short):
        regs = (r["vgpr_count"] or 0) + (r["agpr_count"] or 0)
        w = min(8, 512 // max(regs, 1)) if regs else 8
        print(f"  {n[:58]:58s} {r['vgpr_count']:5d} {r['agpr_count']:5d} {r['sgpr_count']:5d} {r['vgpr_spill_count']:8d} "
              f"{r['sgpr_spill_count']:8d} {r['private_segment_fixed_size']:9d} {r['group_segment_fixed_size']:7d} "
              f"{r['max_flat_workgroup_size']:6d} {w:10d}")


if __name__ == "__main__":
    main()
