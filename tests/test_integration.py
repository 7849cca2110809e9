"""INTEGRATION.md section 1, as a maintainer would apply it: the drop-in blocks are spliced into a
COPY of the reference's src/rt.cpp (in a temporary directory; /root/reference is never written)
in place of main()'s framebuffer, OpenMP loop, clamp and PPM writer (src/rt.cpp:762-820), and the
result is compiled against the reference's own headers and linked against libvpt.so (oracle/dropin.py).
Needs the reference checkout (this container only) and clang++; skipped elsewhere.  The programs
built by __graft_entry__.build() (oracle/_ref/rt_vpt, rt_vpt_multi) are RUN on the GPU by
tests/test_gpu_multi.py."""
import os
import shutil
import subprocess

import pytest

from oracle import dropin

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
PKG = os.path.join(ROOT, "minimal_volumetric_path_tracer_amd")

pytestmark = pytest.mark.skipif(
    not (os.path.isfile(os.path.join(REF, "src", "rt.cpp")) and os.path.exists(CLANG)
         and os.path.exists(os.path.join(PKG, "libvpt.so"))),
    reason="needs the reference checkout, clang++ and a built libvpt.so")


_block, _spliced = dropin.block, dropin.spliced


def _compile(tmp_path, source: str, extra=()):
    exe = tmp_path / "rt_vpt"
    r = dropin.compile_program(source, str(exe), str(tmp_path), extra, opt="-O0")
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
    exe = _compile(tmp_path, _spliced(_block("multi"), "#include <hip/hip_runtime_api.h>\n"), dropin.MULTI_FLAGS)
    nm = subprocess.run(["nm", "-D", "--undefined-only", str(exe)], capture_output=True, text=True).stdout
    assert "vpt_render_multi" in nm


def test_reference_tree_untouched():
    """the splice works on a copy: the reference's rt.cpp still has its own loop"""
    src = open(os.path.join(REF, "src", "rt.cpp"), encoding="utf-8", errors="surrogateescape").read()
    assert "#pragma omp parallel for" in src and "vpt.h" not in src
    assert shutil.which("nm")
