"""Phase timing of the small-grid conv kernel (csrc/conv3d_sg.hip) from in-kernel
s_memtime stamps.

usage: python tools/sg_stamps.py [CASE ...]   (CASE as in tools/conv_bench.py, W < 32)
needs the diagnostics build (tools/build_ab_lib.sh stamps HEAD STAMPS=1, then
CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1).  Per workgroup:
first DMA (start -> first barrier), chunks, split-K publish / last-arrival
reduce, epilogue; and the spread of workgroup start / end times (realtime
clock, 100 MHz).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-cwdm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import conv_bench  # noqa: E402
from cwdm_hip._lib import lib  # noqa: E402


def one(case):
    spec = conv_bench.CASES[case]
    buf = torch.zeros(4096 * 24, dtype=torch.int64, device="cuda")
    conv_bench.run_case(case, spec, 20, 1)  # warm + event timing of the whole call
    lib().cwdm_debug_conv_stamps(ctypes.c_void_p(buf.data_ptr()))
    conv_bench.run_case(case, spec, 1, 1)
    torch.cuda.synchronize()
    lib().cwdm_debug_conv_stamps(None)
    st = [r for r in buf.view(4096, 24).cpu().tolist() if r[0] != 0]
    # the last launch of run_case wrote the stamps (3 warm-ups + 1 timed, all the same grid)
    n = len(st)
    mean = lambda v: sum(v) / max(len(v), 1)
    print(f"{case}: {n} workgroups; cycles mean / min / max")

    def row(nm, v):
        if v:
            print(f"  {nm:26s} {mean(v):9.0f} {min(v):9d} {max(v):9d}")

    row("first DMA (0 -> 1)", [r[1] - r[0] for r in st])
    nch = [sum(1 for k in range(8) if r[4 + k]) for r in st]
    for c in range(max(nch)):
        row(f"chunk {c}", [r[4 + c] - (r[1] if c == 0 else r[3 + c]) for r in st if r[4 + c]])
    row("MFMA loop (1 -> 12)", [r[12] - r[1] for r in st])
    row("publish (12 -> 13)", [r[13] - r[12] for r in st if r[13]])
    row("last reduce (13 -> 14)", [r[14] - r[13] for r in st if r[14]])
    row("epilogue (12|14 -> 15)", [r[15] - (r[14] or r[12]) for r in st if not r[13] or r[14]])
    row("total (0 -> 15)", [r[15] - r[0] for r in st])
    t0 = min(r[20] for r in st)
    starts = [(r[20] - t0) / 100.0 for r in st]
    ends = [(r[21] - t0) / 100.0 for r in st]
    print(f"  start spread {min(starts):.2f} .. {max(starts):.2f} us; end {min(ends):.2f} .. {max(ends):.2f} us")
    clk = [(r[15] - r[0]) / max(r[21] - r[20], 1) * 0.1 for r in st]
    print(f"  shader clock {mean(clk):.2f} GHz")


def main():
    for case in sys.argv[1:] or ["L3_256_256_gn", "L3_256_256_res", "L4_256_256_gn"]:
        one(case)


if __name__ == "__main__":
    main()
