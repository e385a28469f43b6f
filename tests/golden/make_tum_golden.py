"""Golden vectors for the TUM timestamp association (associate.py).

Run in the dev container (where /root/reference exists): imports the reference's
associate.py, feeds it synthetic rgb/depth lists through its own read_file_list, and stores
the inputs (as text) and its matches in tum_assoc.json.  associate() is Python-2 code
(dict.keys().remove), so the dicts handed to it return list keys; nothing else is changed.
"""
import importlib.util
import json
import os
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/associate.py"


class _ListKeys(dict):
    def keys(self):
        return list(super().keys())


def main():
    spec = importlib.util.spec_from_file_location("ref_associate", REF)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    rng = np.random.default_rng(0)
    cases = []
    for case in range(4):
        t0 = 1305031102.0 + case
        rgb = np.round(t0 + np.arange(120) / 30.0 + rng.normal(0, 0.004, 120), 6)
        dep = np.round(t0 + 0.011 * case + np.arange(120) / 30.0 + rng.normal(0, 0.004, 120), 6)
        keep_r = rng.random(120) > 0.05
        keep_d = rng.random(120) > 0.05
        rgb_txt = "# color images\n# file: 'x.bag'\n# timestamp filename\n" + "".join(
            "%.6f rgb/%.6f.png\n" % (t, t) for t in rgb[keep_r])
        dep_txt = "# depth maps\n" + "".join("%.6f depth/%.6f.png\n" % (t, t) for t in dep[keep_d])
        offset, maxd = [(0.0, 0.02), (0.0, 0.01), (-0.011, 0.02), (0.0, 0.05)][case]
        with tempfile.TemporaryDirectory() as d:
            fr, fd = os.path.join(d, "rgb.txt"), os.path.join(d, "depth.txt")
            open(fr, "w").write(rgb_txt)
            open(fd, "w").write(dep_txt)
            a, b = m.read_file_list(fr), m.read_file_list(fd)
        matches = m.associate(_ListKeys(a), _ListKeys(b), offset, maxd)
        cases.append(dict(rgb=rgb_txt, depth=dep_txt, offset=offset, max_difference=maxd,
                          matches=[[x, y] for x, y in matches]))
    json.dump(cases, open(os.path.join(HERE, "tum_assoc.json"), "w"))
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
