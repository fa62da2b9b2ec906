"""The diagnostic builds kept in the kernel sources (OMR_BWD_COUNT, OMR_STAMPS; OMR_LB_SPIN_MAX=0 is built by the
default target for tests/test_gpu_errors.py) must keep compiling: `make variants` cross-compiles each for gfx950.
No GPU needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "omnigs-fork_amd", "csrc")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_diagnostic_variants_compile():
    r = subprocess.run(["make", "-s", "-j4", "-C", CSRC, "variants"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("render_bwd_count.o", "render_bwd_stamps.o", "render_fwd_stamps.o"):
        assert os.path.getsize(os.path.join(ROOT, "omnigs-fork_amd", "lib", "obj", "variants", name)) > 0
