"""Host-side C++ test of the GEMM grid planning the gfx950 kernels use (csrc/tile_plan.h: XCD remap
bijectivity, split-tail coverage and planner rules), built with AddressSanitizer and
UndefinedBehaviorSanitizer (SURVEY.md §5 race detection / sanitizers: host code; GPU sanitizers are
not available on the MI355X pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_tile_plan.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_tile_plan_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "test_tile_plan")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", SRC, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
