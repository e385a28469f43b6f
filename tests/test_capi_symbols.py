"""The C-ABI library loads (no GPU needed) and exports every entry point include/*.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "coeb-slam_amd", "lib", "libcoeb_front.so")


def declared():
    txt = open(os.path.join(ROOT, "include", "coeb_front.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(coeb_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "coeb-slam_amd", "csrc")])
    return ctypes.CDLL(LIB)


def test_header_declares_abi():
    d = declared()
    assert "coeb_extract" in d and "coeb_match_lastframe" in d and "coeb_create" in d


def test_every_declared_symbol_exported(lib):
    missing = [s for s in declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_mirror_lists_abi():
    import coeb_front
    assert sorted(coeb_front.ABI_SYMBOLS) == declared()


def test_descriptor_distance_cpu_entry(lib):
    import numpy as np
    a = np.arange(32, dtype=np.uint8)
    b = a[::-1].copy()
    d = lib.coeb_descriptor_distance(a.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p))
    assert d == int(np.unpackbits(a ^ b).sum())


def test_no_gpu_fails_loudly(lib):
    """Without a gfx950 device coeb_create returns NULL with a message; no CPU fallback."""
    if lib.coeb_device_count() > 0:
        pytest.skip("a GPU is visible")
    import coeb_front
    with pytest.raises(coeb_front.CoebError):
        coeb_front.Context()


def test_boxes_from_int64_host_only():
    """coeb_boxes_from_int64 (ros_rgbd.cc:106-115 int64 -> float) is host code: no GPU needed."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
    import coeb_front
    b = np.array([[10, 20, 300, 400], [-5, 0, 2 ** 40, 7]], np.int64)
    assert np.array_equal(coeb_front.boxes_from_ros(b), b.astype(np.float32))


def test_abi_version_matches_header(lib):
    txt = open(os.path.join(ROOT, "include", "coeb_front.h")).read()
    want = int(re.search(r"#define COEB_ABI_VERSION (\d+)", txt).group(1))
    assert lib.coeb_abi_version() == want
    import sys
    sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
    import coeb_front
    assert coeb_front.ABI_VERSION == want      # the ctypes argtypes are written for this header


def test_last_error_is_per_thread(lib):
    """coeb_last_error(NULL) is thread-local: ranks of `bench.py --gpus N` (one host thread per
    device) fail concurrently without racing on one std::string.  Here every thread alternates two
    coeb_create failures that need no GPU (bad arguments / no usable device) and must read back
    exactly its own message each time."""
    import threading

    class Params(ctypes.Structure):
        _fields_ = [("nfeatures", ctypes.c_int), ("scale_factor", ctypes.c_float), ("nlevels", ctypes.c_int),
                    ("ini_th", ctypes.c_int), ("min_th", ctypes.c_int)]

    lib.coeb_create.restype = ctypes.c_void_p
    lib.coeb_create.argtypes = [ctypes.POINTER(Params), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.coeb_last_error.restype = ctypes.c_char_p
    lib.coeb_last_error.argtypes = [ctypes.c_void_p]
    prm = Params(1000, 1.2, 8, 20, 7)
    if lib.coeb_create(ctypes.byref(prm), 0, 640, 480, 1):
        pytest.skip("a usable device is present: the no-device failure cannot be provoked")
    bad = []

    def body(t):
        for i in range(300):
            invalid = (i + t) % 2 == 0
            h = lib.coeb_create(ctypes.byref(prm), 0, 0 if invalid else 640, 480, 1)
            assert not h
            msg = lib.coeb_last_error(None).decode()
            if invalid != ("invalid arguments" in msg):
                bad.append((t, i, msg))

    ths = [threading.Thread(target=body, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not bad, bad[:3]
