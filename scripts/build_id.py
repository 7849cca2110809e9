"""Build id of libvpt.so: sha256 over the native sources (path + NUL + bytes, sorted) and the compile
flags, first 16 hex digits.  The Makefile bakes it into the library (vpt_build_id()); the CPU test
tests/test_build_id.py recomputes it from the tree, so a stale prebuilt .so is caught.
usage: python scripts/build_id.py "<flags>"   (run from anywhere)"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join("minimal_volumetric_path_tracer_amd", "csrc")


def source_files():
    names = [os.path.join(CSRC, f) for f in os.listdir(os.path.join(ROOT, CSRC))
             if f.endswith((".h", ".hip", ".cpp")) or f == "Makefile"]
    return sorted(names + [os.path.join("include", "vpt.h")])


def build_id(flags: str) -> str:
    h = hashlib.sha256()
    for rel in source_files():
        h.update(rel.replace(os.sep, "/").encode() + b"\0")
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
    h.update(b"flags\0" + " ".join(flags.split()).encode())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(build_id(sys.argv[1] if len(sys.argv) > 1 else ""))
