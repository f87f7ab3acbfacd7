"""The product build refuses the timing-only ablation switches.

SLAM_ABL_* (and SLAM_NO_WINX, SLAM_KABSCH_ALL) remove work from the ICP kernel
to time its phases and give wrong results.  The
in-tree library's flags (csrc/Makefile, -DSLAMHIP_PRODUCT_BUILD) must turn any
of them into a compile error; the A/B builds (tools/ab_build.sh) add
SLAM_TIMING_ONLY.  Host-side syntax check with hipcc, no GPU needed."""
import os
import shlex
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from conftest import PKG

CSRC = os.path.join(PKG, "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["SLAM_ABL_SUMS", "SLAM_ABL_GROUP", "SLAM_ABL_CERT", "SLAM_ABL_STAGE2X", "SLAM_NO_WINX", "SLAM_KABSCH_ALL"]


def product_flags():
    out = subprocess.run(["make", "-s", "--no-print-directory", "-C", CSRC, "print-flags"], check=True,
                         capture_output=True, text=True).stdout
    return shlex.split(out)


def syntax(extra):
    cmd = [HIPCC, "-fsyntax-only"] + [f for f in product_flags() if f not in ("-O3",)] + extra + ["icp_kernels.hip"]
    return subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_product_build_refuses_ablation_flags():
    assert "-DSLAMHIP_PRODUCT_BUILD" in product_flags()
    with ThreadPoolExecutor(len(FLAGS)) as ex:
        runs = list(ex.map(lambda f: syntax([f"-D{f}"]), FLAGS))
    for f, r in zip(FLAGS, runs):
        assert r.returncode != 0, f
        assert "timing-only" in r.stderr, (f, r.stderr[-400:])


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_timing_only_build_is_still_refused_in_product_flags():
    r = syntax(["-DSLAM_TIMING_ONLY", "-DSLAM_ABL_GROUP"])
    assert r.returncode != 0 and "product build" in r.stderr
