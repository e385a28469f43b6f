"""Pack the reference's own TUM association outputs (Examples/RGB-D/associations/*.txt, the
output of associate.py:49-102 on the TUM sequences, 18,520 rgb/depth stamp pairs) into
tests/golden/tum_assoc_files.npz, one compressed byte array per file, so the test that re-derives
them (tests/test_oracle_kat.py::test_tum_association_reference_files) runs without /root/reference.

    python tests/golden/make_tum_assoc_files.py [/root/reference]
"""
import glob
import os
import sys

import numpy as np

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
files = sorted(glob.glob(os.path.join(ref, "Examples", "RGB-D", "associations", "*.txt")))
assert files, "no association files under %s" % ref
arrays = {os.path.basename(f)[:-4]: np.frombuffer(open(f, "rb").read(), np.uint8) for f in files}
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tum_assoc_files.npz")
np.savez_compressed(out, **arrays)
print("%d files, %d bytes -> %s (%d bytes)" % (len(arrays), sum(a.size for a in arrays.values()), out,
                                               os.path.getsize(out)))
