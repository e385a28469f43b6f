"""Runtime switches of the shipped library: the library reads the environment
only through coeb_switch() / coeb_experiment() (csrc/coeb_capi.hip); every product switch is on the
kSwitches list and is set by at least one GPU test, and experiment switches are read only under
COEB_EXPERIMENTS=1.  Also: the one -Wpass-failed diagnostic that coeb_flow.hip suppresses is the
expected k_fm<128> occupancy target and nothing else (an unroll or other pass failure would show)."""
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "coeb-slam_amd", "csrc")


def _sources():
    return {os.path.basename(p): open(p).read() for p in sorted(glob.glob(os.path.join(CSRC, "*.hip")) +
                                                                 glob.glob(os.path.join(CSRC, "*.hpp")) +
                                                                 glob.glob(os.path.join(CSRC, "*.cpp")))}


def test_environment_read_only_through_the_switch_helpers():
    src = _sources()
    calls = [(f, m.start()) for f, s in src.items() for m in re.finditer(r"\bgetenv\s*\(", s)]
    assert len(calls) == 3 and {f for f, _ in calls} == {"coeb_capi.hip"}, calls
    capi = src["coeb_capi.hip"]
    for _, pos in calls:
        fn = capi.rfind("const char* coeb_", 0, pos)
        assert capi[fn:fn + 40].startswith(("const char* coeb_switch(", "const char* coeb_experiment(")), \
            capi[fn:fn + 60]


def test_every_product_switch_is_listed_and_tested():
    src = _sources()
    listed = re.findall(r'^\s*"(COEB_[A-Z_0-9]+)",', src["coeb_capi.hip"].split("kSwitches[] = {", 1)[1].split("};", 1)[0],
                        re.M)
    used = {n for s in src.values() for n in re.findall(r'coeb_switch\("(COEB_[A-Z_0-9]+)"\)', s)}
    assert used and used <= set(listed), used - set(listed)
    tests = "".join(open(p).read() for p in glob.glob(os.path.join(ROOT, "tests", "test_gpu*.py")))
    untested = [n for n in listed if n not in tests]
    assert not untested, "product switches no GPU test sets: %s" % untested


def test_k_fm_pass_failed_suppression_hides_only_the_occupancy_target(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    s = open(os.path.join(CSRC, "coeb_flow.hip")).read()
    assert s.count('#pragma clang diagnostic ignored "-Wpass-failed"') == 1
    f = tmp_path / "flow_unsuppressed.hip"
    f.write_text(s.replace('#pragma clang diagnostic ignored "-Wpass-failed"', ""))
    out = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
                          "-Wall", "-Wno-unused-function", "-I", CSRC, "-c", str(f), "-o", str(tmp_path / "f.o")],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    warns = [l for l in out.stderr.splitlines() if "warning:" in l]
    assert len(warns) == 1, warns
    assert "k_fmILi128" in warns[0] and "amdgpu-waves-per-eu" in warns[0] and "-Wpass-failed" in warns[0], warns[0]
