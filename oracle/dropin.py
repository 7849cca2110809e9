"""TEST INFRASTRUCTURE ONLY -- INTEGRATION.md section 1 applied as a maintainer would: the drop-in
blocks are spliced into a COPY of the reference's src/rt.cpp (in a temporary directory;
/root/reference is never written, and the spliced source is never kept) in place of main()'s
framebuffer, OpenMP loop, clamp and PPM writer (src/rt.cpp:762-820), compiled against the
reference's own headers and linked against libvpt.so.

    python oracle/dropin.py        # -> oracle/_ref/rt_vpt, oracle/_ref/rt_vpt_multi

Built in this container only (it needs the reference checkout); the binaries travel to the GPU
box with oracle/_ref/, where tests/test_gpu_multi.py runs them.  tests/test_integration.py checks
the splice and the link here."""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference"
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
PKG = os.path.join(ROOT, "minimal_volumetric_path_tracer_amd")
MULTI_FLAGS = ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]


def available() -> bool:
    return (os.path.isfile(os.path.join(REF, "src", "rt.cpp")) and os.path.exists(CLANG)
            and os.path.exists(os.path.join(PKG, "libvpt.so")))


def block(name: str) -> str:
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"<!-- dropin:%s -->\s*```cpp\n(.*?)```" % name, text, re.S)
    if not m:
        raise ValueError(f"INTEGRATION.md has no dropin:{name} block")
    return m.group(1)


def spliced(body: str, extra_top: str = "") -> str:
    src = open(os.path.join(REF, "src", "rt.cpp"), encoding="utf-8", errors="surrogateescape").read()
    start = src.index("Color *pixelColors = new Color[w * h];")
    end = src.index("delete[] pixelColors;") + len("delete[] pixelColors;")
    return extra_top + block("top") + src[:start] + body + src[end:]


def compile_program(source: str, exe: str, workdir: str, extra=(), opt="-O2") -> subprocess.CompletedProcess:
    cpp = os.path.join(workdir, "rt_vpt.cpp")
    with open(cpp, "w", encoding="utf-8", errors="surrogateescape") as f:
        f.write(source)
    cmd = [CLANG, "-std=c++20", opt, "-w", "-include", os.path.join(HERE, "ref_prelude.h"),
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(REF, "include"), cpp,
           os.path.join(REF, "include", "Sphere.cpp"), os.path.join(REF, "include", "Vector.cpp"),
           os.path.join(REF, "include", "Ray.cpp"), "-L", PKG, "-lvpt", "-Wl,-rpath,$ORIGIN/../../minimal_volumetric_path_tracer_amd",
           "-Wl,-rpath,/opt/rocm/lib/llvm/lib", "-L/opt/rocm/lib/llvm/lib", *extra, "-o", exe]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600)


def build() -> None:
    out = os.path.join(HERE, "_ref")
    os.makedirs(out, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        for name, src, extra in (("rt_vpt", spliced(block("body")), []),
                                 ("rt_vpt_multi", spliced(block("multi"), "#include <hip/hip_runtime_api.h>\n"),
                                  MULTI_FLAGS)):
            r = compile_program(src, os.path.join(out, name), td, extra)
            if r.returncode != 0:
                raise RuntimeError(f"{name}: {r.stderr[-2000:]}")


if __name__ == "__main__":
    if not available():
        sys.exit("needs /root/reference, clang++ and a built libvpt.so")
    build()
    print("built oracle/_ref/rt_vpt, oracle/_ref/rt_vpt_multi")
