"""Build provenance: the libvpt.so in the tree carries the id of the sources and flags it was built
from (csrc/Makefile bakes scripts/build_id.py's hash in), so a stale prebuilt library is caught on
the CPU before any GPU run uses it."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import build_id as bid  # noqa: E402

import minimal_volumetric_path_tracer_amd as vpt  # noqa: E402


def _make_flags() -> str:
    """BUILD_FLAGS as the Makefile expands it (make -pn prints the variable database)."""
    out = subprocess.run(["make", "-pn", "-C", os.path.join(ROOT, "minimal_volumetric_path_tracer_amd", "csrc")],
                         capture_output=True, text=True).stdout
    return re.search(r"^BUILD_FLAGS := (.*)$", out, re.M).group(1)


def test_library_build_id_matches_tree():
    got = vpt.build_id()
    assert re.fullmatch(r"[0-9a-f]{16}", got), got
    assert got == bid.build_id(_make_flags()), "libvpt.so was built from other sources or flags: rebuild it"


def test_build_id_changes_with_flags():
    assert bid.build_id("-O3") != bid.build_id("-O2")
