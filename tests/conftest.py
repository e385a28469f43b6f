"""Test configuration.  `-m "not gpu"`: oracle KATs, golden fixtures, host logic, C-ABI
exports, gloo multi-rank logic (runs in the dev container).  `-m gpu`: HIP-vs-oracle parity
through the C-ABI on an MI355X.  GPU tests never import torch.cuda: the torch wheel's
bundled HIP runtime cannot share a process with libcoeb_front.so."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "coeb-slam_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libcoeb_front.so")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O
    if not os.path.exists(O.LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return O


@pytest.fixture(scope="session")
def ctx():
    from coeb_front import Context
    c = Context(max_width=1280, max_height=960, max_batch=16)
    yield c
    c.close()
