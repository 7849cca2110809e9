"""Every compile-time arm the release build does not take still compiles: the
kept structural knob (VPT_KILL_RINGS=0, the pool without kill-predicting rings), the forms the round-6
changes replaced, and the debug / measurement builds (section timers, scheduler statistics and
timelines, the round-1 wave kernel behind VPT_DEBUG_ENV, a VPT_DUP build).
A device-side syntax and template-instantiation check of csrc/vpt_kernels.hip for gfx950 -- seconds,
no GPU; the A/B builds themselves go through scripts/build_variant.sh."""
import os
import shutil
import subprocess

import pytest

HIPCC = "/opt/rocm/bin/hipcc"
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "minimal_volumetric_path_tracer_amd",
                    "csrc")

ARMS = {
    "no_kill_rings": ["-DVPT_KILL_RINGS=0"],
    "sections": ["-DVPT_SECTIONS=1"],
    "sections_no_kill_rings": ["-DVPT_SECTIONS=1", "-DVPT_KILL_RINGS=0"],
    "pool_stats": ["-DVPT_POOL_DEBUG=1"],
    "pool_timeline": ["-DVPT_POOL_DEBUG=2"],
    "debug_env": ["-DVPT_DEBUG_ENV=1"],
    "params_in_sgprs": ["-DVPT_P_KARG=0"],  # launch parameters held for the whole kernel (pre-round-5 form)
    # the round-6 changes off (the forms they replaced, for A/B): branchy sphere-test update outside the
    # det >= 0 branch, branchy frames, exec-masked rare paths, plain divisions, general cone acos/cos
    "round6_off": ["-DVPT_TAKE_SEL=0", "-DVPT_TAKE_IN=0", "-DVPT_FRAME_SEL=0", "-DVPT_RARE_BALLOT=0",
                   "-DVPT_DIV_SHARE=0", "-DVPT_ACOS_CONE=0", "-DVPT_COS_ACOS_C=0", "-DVPT_FRAME_CSE=0",
                   "-DVPT_MIS_REUSE=0", "-DVPT_PL_REUSE=0", "-DVPT_ISECT_CLASS=0", "-DVPT_ISECT_VIDX=0", "-DVPT_ISECT_ZERO=0", "-DVPT_MARCH_REUSE=0",
                   "-DVPT_SS_FUSE=0"],
    "dup_sections": ["-DVPT_DUP=3"],  # a VPT_DUP measurement build (scripts/dup_pmc.sh)
}


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="hipcc not installed")
@pytest.mark.parametrize("arm", sorted(ARMS))
def test_knob_arm_compiles(arm):
    cmd = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off", "-fsyntax-only", "--cuda-device-only",
           "-Wno-unused-command-line-argument", "-DVPT_MIS_TU=0"] + ARMS[arm] + ["vpt_kernels.hip"]
    r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
