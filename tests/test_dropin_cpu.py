"""The drop-in claim, checked by the compiler: the reference's own test and
CLI sources -- /root/reference/tests/{ials,ialspp,erm_mf,cvar_mf,safer2,
safer2pp}_test.cc and /root/reference/tools/run_model.cc (with the CLI11
header the reference vendors at tools/CLI11) -- compile with -fsyntax-only
against the product's headers (safer2-recommender_amd/include, the
reference class names and constructor signatures, include/frecsys_hip.h)
plus the tests-only gtest / glog / fmt / Eigen stand-ins under tests/shim.

Compile only: -fsyntax-only writes no object, so nothing built from the
reference exists, let alone travels to the GPU box.  Skipped where the
reference tree is absent (the GPU box).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
SOURCES = [f"tests/{m}_test.cc" for m in ("ials", "ialspp", "erm_mf", "cvar_mf", "safer2",
                                           "safer2pp")] + ["tools/run_model.cc"]

pytestmark = pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("g++") is None,
                                reason="reference tree or g++ absent")


@pytest.mark.parametrize("src", SOURCES)
def test_reference_source_compiles_against_product_headers(src):
    path = os.path.join(REF, src)
    assert os.path.exists(path), path
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-Wno-deprecated-declarations",
           "-I", os.path.join(ROOT, "tests", "shim"),
           "-I", os.path.join(ROOT, "safer2-recommender_amd", "include"),
           "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(REF, "tools"),
           path]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-6000:]
