"""INTEGRATION.md section 1, as a maintainer would apply it: the drop-in blocks are spliced into a
COPY of the reference's src/rt.cpp (in a temporary directory; /root/reference is never written)
in place of main()'s framebuffer, OpenMP loop, clamp and PPM writer (src/rt.cpp:762-820), and the
result is compiled against the reference's own headers and linked against libvpt.so.  Needs the
reference checkout (this container only) and clang++; skipped elsewhere.  Running the program
needs a GPU: the `vpt` program, which makes the same calls, is run by tests/test_gpu_multi.py."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
PKG = os.path.join(ROOT, "minimal_volumetric_path_tracer_amd")

pytestmark = pytest.mark.skipif(
    not (os.path.isfile(os.path.join(REF, "src", "rt.cpp")) and os.path.exists(CLANG)
         and os.path.exists(os.path.join(PKG, "libvpt.so"))),
    reason="needs the reference checkout, clang++ and a built libvpt.so")


def _block(name: str) -> str:
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"<!-- dropin:%s -->\s*```cpp\n(.*?)```" % name, text, re.S)
    assert m, f"INTEGRATION.md has no dropin:{name} block"
    return m.group(1)


def _spliced(body: str, extra_top: str = "") -> str:
    src = open(os.path.join(REF, "src", "rt.cpp"), encoding="utf-8", errors="surrogateescape").read()
    start = src.index("Color *pixelColors = new Color[w * h];")
    end = src.index("delete[] pixelColors;") + len("delete[] pixelColors;")
    return extra_top + _block("top") + src[:start] + body + src[end:]


def _compile(tmp_path, source: str, extra=()):
    cpp = tmp_path / "rt_vpt.cpp"
    cpp.write_text(source, encoding="utf-8", errors="surrogateescape")
    exe = tmp_path / "rt_vpt"
    cmd = [CLANG, "-std=c++20", "-O0", "-w", "-include", os.path.join(ROOT, "oracle", "ref_prelude.h"),
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(REF, "include"), str(cpp),
           os.path.join(REF, "include", "Sphere.cpp"), os.path.join(REF, "include", "Vector.cpp"),
           os.path.join(REF, "include", "Ray.cpp"), "-L", PKG, "-lvpt", f"-Wl,-rpath,{PKG}",
           "-Wl,-rpath,/opt/rocm/lib/llvm/lib", "-L/opt/rocm/lib/llvm/lib", *extra, "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def test_dropin_single_gpu_compiles_and_links(tmp_path):
    exe = _compile(tmp_path, _spliced(_block("body")))
    nm = subprocess.run(["nm", "-D", "--undefined-only", str(exe)], capture_output=True, text=True).stdout
    for sym in ("vpt_context_create", "vpt_set_scene", "vpt_render", "vpt_write_ppm"):
        assert sym in nm, sym
    src = (tmp_path / "rt_vpt.cpp").read_text(encoding="utf-8", errors="surrogateescape")
    assert "#pragma omp parallel for" not in src.split("int main(")[1]  # the OpenMP loop is gone
    assert "iterativeVPTracerFree(Ray(camera.o" not in src.split("int main(")[1]


def test_dropin_multi_gpu_compiles_and_links(tmp_path):
    exe = _compile(tmp_path, _spliced(_block("multi"), "#include <hip/hip_runtime_api.h>\n"),
                   ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,/opt/rocm/lib"])
    nm = subprocess.run(["nm", "-D", "--undefined-only", str(exe)], capture_output=True, text=True).stdout
    assert "vpt_render_multi" in nm


def test_reference_tree_untouched():
    """the splice works on a copy: the reference's rt.cpp still has its own loop"""
    src = open(os.path.join(REF, "src", "rt.cpp"), encoding="utf-8", errors="surrogateescape").read()
    assert "#pragma omp parallel for" in src and "vpt.h" not in src
    assert shutil.which("nm")
