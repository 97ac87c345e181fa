"""GPU: the fast correctly-rounded helpers (csrc/cr_math.h) equal the compiler's IEEE sqrt, reciprocal
and division bit for bit over their domains (exhaustive for sqrt and reciprocal, and for the general
1/sqrt over all 2^32 inputs)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cr_math_bit_exact(tmp_path):
    exe = tmp_path / "crmath_check"
    csrc = os.path.join(ROOT, "simple-path-tracer_amd", "csrc")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                    "-I", csrc, os.path.join(ROOT, "tests", "hip", "crmath_check.hip"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count(" 0 mismatches") == 5, res.stdout
