"""Phase timing of the second-generation output head (conv3d_head.hip head2_kernel)
from in-kernel s_memtime stamps: per tile of a workgroup's first z column, how
long the MFMA waves computed and ran the epilogue, when the fill waves had the
next planes loaded + transformed and stored, and when each side reached the
tile barrier.

usage: CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 python tools/head_stamps.py [CASE]
(the library built with make STAMPS=1; CASE as in tools/conv_bench.py)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-cwdm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import conv_bench  # noqa: E402
from cwdm_hip._lib import lib  # noqa: E402


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "L0_64_8_out"
    spec = conv_bench.CASES[case]
    nwg = torch.cuda.get_device_properties(0).multi_processor_count
    buf = torch.zeros(nwg * 64, dtype=torch.int64, device="cuda")
    conv_bench.run_case(case, spec, 3, 1)  # warm
    lib().cwdm_debug_conv_stamps(ctypes.c_void_p(buf.data_ptr()))
    conv_bench.run_case(case, spec, 1, 1)
    torch.cuda.synchronize()
    lib().cwdm_debug_conv_stamps(None)
    report(case, buf, nwg)


def report(case, buf, nwg):
    st = [r for r in buf.view(nwg, 64).cpu().tolist() if r[0] != 0]
    mean = lambda v: sum(v) / max(len(v), 1)  # noqa: E731
    print(f"{case}: {len(st)} workgroups; cycles from the previous tile barrier, mean (min / max)")
    print(f"  prologue (start -> MFMA waves past B0) {mean([r[1] - r[0] for r in st]):8.0f}")
    for k in range(8):
        if not all(r[1 + 3 * k] and r[3 + 3 * k] for r in st):
            break
        t0 = [r[1 + 3 * k] for r in st]
        cols = [("MFMAs", 2 + 3 * k), ("MFMA at barrier", 3 + 3 * k), ("fill stored", 33 + 3 * k),
                ("fill loaded+transformed", 32 + 3 * k), ("fill at barrier", 34 + 3 * k)]
        parts = []
        for name, idx in cols:
            v = [r[idx] - a for r, a in zip(st, t0) if r[idx]]
            if v:
                parts.append(f"{name} {mean(v):6.0f} ({min(v)}/{max(v)})")
        print(f"  tile {k}: " + "  ".join(parts))
    tot = [r[62] - r[0] for r in st if r[62]]
    clk = [(r[62] - r[0]) / max(r[61] - r[60], 1) * 0.1 for r in st if r[61] and r[62]]
    if clk:
        print(f"  first column {mean(tot):.0f} cycles; shader clock ~{mean(clk):.2f} GHz "
              "(s_memtime vs s_memrealtime at 100 MHz)")


if __name__ == "__main__":
    main()
