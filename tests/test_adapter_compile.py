"""The drop-in C++ adapters (coeb-slam_amd/adapter/) compile against reference-shaped types.

Compile-only (-fsyntax-only) with a minimal OpenCV stand-in under tests/adapter_shim: the
signatures mirrored are ORBextractor.h:44-128 and ORBmatcher.h:52 / ORBmatcher.cc:1329."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_adapters_compile():
    shim = os.path.join(ROOT, "tests", "adapter_shim")
    cmd = ["g++", "-std=c++14", "-fsyntax-only", "-Wall", "-Werror",
           "-I", shim, "-I", os.path.join(ROOT, "coeb-slam_amd", "adapter"), "-I", os.path.join(ROOT, "include"),
           os.path.join(shim, "adapter_tu.cpp")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
