"""Generate tests/golden/pywt_haar3d_wavedec2.npz: multi-level Haar
(pywt.wavedecn / waverecn, level 2, 'periodization') for the multi-level
DWT of BASELINE config 5 (TEST INFRASTRUCTURE; same library and key mapping
as gen_pywt_golden.py: pywt 'a'/'d' per axis (D, H, W) = reference L/H).

Run with:  /opt/conda/bin/python3.9 oracle/gen_pywt_wavedec_golden.py
"""
import os
import sys

import numpy as np
import pywt

BANDS = ("LLH", "LHL", "LHH", "HLL", "HLH", "HHL", "HHH")


def main(out):
    rng = np.random.RandomState(1)
    arrs = {}
    for n, shp in enumerate([(8, 12, 16), (16, 16, 16), (4, 8, 12)]):
        x = rng.standard_normal(shp)
        coeffs = pywt.wavedecn(x, "haar", mode="periodization", level=2)
        arrs[f"x{n}"] = x
        arrs[f"x{n}_L2_LLL"] = coeffs[0]
        for lev, d in ((2, coeffs[1]), (1, coeffs[2])):
            for b in BANDS:
                arrs[f"x{n}_L{lev}_{b}"] = d["".join("a" if c == "L" else "d" for c in b)]
        arrs[f"x{n}_rec"] = pywt.waverecn(coeffs, "haar", mode="periodization")
    arrs["pywt_version"] = np.array(pywt.__version__)
    np.savez(out, **arrs)
    print("wrote", out, "pywt", pywt.__version__)


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "..", "tests", "golden", "pywt_haar3d_wavedec2.npz"))
