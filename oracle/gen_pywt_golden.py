"""Generate tests/golden/pywt_haar3d.npz from PyWavelets (TEST INFRASTRUCTURE).

The reference takes its Haar taps from ``pywt.Wavelet('haar')``
(DWT_IDWT/DWT_IDWT_layer.py:451-457, pinned PyWavelets==1.4.1 in
environment.yml:13).  PyWavelets 1.1.1 is installed under /opt/conda's
python3.9 in this image (not importable from the main interpreter), and its
Haar filter bank is unchanged between 1.1.1 and 1.4.1.  This script records
``pywt.dwtn`` / ``pywt.idwtn`` outputs for a few seeded volumes so the
oracle's wavelet restatement is pinned to the library the reference uses.

Run with:  /opt/conda/bin/python3.9 oracle/gen_pywt_golden.py
pywt key letters index axes in order (axis0=D, axis1=H, axis2=W); 'a' is the
low pass (L) and 'd' the high pass (H), so reference band LHL == pywt 'ada'.
"""
import os
import sys

import numpy as np
import pywt

BANDS = ("LLL", "LLH", "LHL", "LHH", "HLL", "HLH", "HHL", "HHH")


def main(out):
    w = pywt.Wavelet("haar")
    rec = {"rec_lo": np.array(w.rec_lo), "rec_hi": np.array(w.rec_hi),
           "dec_lo": np.array(w.dec_lo), "dec_hi": np.array(w.dec_hi)}
    rng = np.random.RandomState(0)
    shapes = [(2, 2, 2), (4, 6, 8), (8, 8, 8), (6, 10, 4), (16, 12, 14)]
    arrs = dict(rec)
    for n, shp in enumerate(shapes):
        x = rng.standard_normal(shp).astype(np.float64)
        coeffs = pywt.dwtn(x, "haar", mode="periodization")
        arrs[f"x{n}"] = x
        for b in BANDS:
            key = "".join("a" if c == "L" else "d" for c in b)
            arrs[f"x{n}_{b}"] = coeffs[key]
        arrs[f"x{n}_rec"] = pywt.idwtn(coeffs, "haar", mode="periodization")
    arrs["pywt_version"] = np.array(pywt.__version__)
    np.savez(out, **arrs)
    print("wrote", out, "pywt", pywt.__version__)


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "..", "tests", "golden", "pywt_haar3d.npz"))
