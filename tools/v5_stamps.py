"""Phase timing of the warp-specialised conv (conv3d_v5.hip) from in-kernel
s_memtime stamps: per chunk, how long the MFMA waves computed, how long they
then waited at the chunk barrier, and when the helper waves arrived there.

usage: CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 python tools/v5_stamps.py CASE
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
    case = sys.argv[1] if len(sys.argv) > 1 else "L0_64_64_gn"
    spec = conv_bench.CASES[case]
    nwg = torch.cuda.get_device_properties(0).multi_processor_count
    buf = torch.zeros(nwg * 64, dtype=torch.int64, device="cuda")
    conv_bench.run_case(case, spec, 3, 1)  # warm
    lib().cwdm_debug_conv_stamps(ctypes.c_void_p(buf.data_ptr()))
    conv_bench.run_case(case, spec, 1, 1)
    torch.cuda.synchronize()
    lib().cwdm_debug_conv_stamps(None)
    st = [r for r in buf.view(nwg, 64).cpu().tolist() if r[0] != 0]
    mean = lambda v: sum(v) / max(len(v), 1)  # noqa: E731
    print(f"{case}: {len(st)} workgroups; cycles, mean over workgroups (min / max)")
    if all(r[55] for r in st):
        print(f"  apply-ahead prologue (entry -> start) {mean([r[0] - r[55] for r in st]):8.0f}"
              f" ({min(r[0] - r[55] for r in st)}/{max(r[0] - r[55] for r in st)});"
              f" helper 0 waiting on range counters {mean([r[56] for r in st]):8.0f} ({max(r[56] for r in st)} max)")
    print(f"  prologue (start -> past B0)   {mean([r[1] - r[0] for r in st]):8.0f}")
    for k in range(16):
        if not all(r[2 + k] for r in st):
            break
        prev = [r[1] if k == 0 else r[18 + k - 1] for r in st]
        comp = [r[2 + k] - p for r, p in zip(st, prev)]
        wait = [r[18 + k] - r[2 + k] for r in st]
        hlp = [r[34 + k] - p for r, p in zip(st, prev)]
        print(f"  chunk {k:2d}: MFMA {mean(comp):7.0f} ({min(comp)}/{max(comp)})  barrier wait {mean(wait):6.0f}"
              f" ({min(wait)}/{max(wait)})  helper at barrier {mean(hlp):7.0f} ({min(hlp)}/{max(hlp)})")
    tot = [r[52] - r[0] for r in st if r[52]]
    clk = [(r[52] - r[0]) / max(r[51] - r[50], 1) * 0.1 for r in st if r[51] and r[52]]
    print(f"  total {mean(tot):.0f} cycles; shader clock ~{mean(clk):.2f} GHz (helper end vs MFMA-wave realtime)")


if __name__ == "__main__":
    main()
