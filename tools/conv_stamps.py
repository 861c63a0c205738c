"""Phase timing of the DMA-staged conv kernel from in-kernel s_memtime stamps.

usage: python tools/conv_stamps.py CASE   (CASE as in tools/conv_bench.py)
needs the diagnostics build: touch csrc/conv3d_v4.hip && make -C fast-cwdm_amd/csrc STAMPS=1
Per workgroup: prologue (start -> first barrier), per-chunk time, epilogue
(last chunk barrier -> end); and how the workgroups sharing a CU overlap.
"""
import collections
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
    case = sys.argv[1] if len(sys.argv) > 1 else "L0_64_64_nogn"
    spec = conv_bench.CASES[case]
    n, cout = spec[0], spec[3]
    nblk = (n // 32) * (n // 4) * (n // 4) * (cout // 64)
    # persistent grid: CWDM_V4_GRID_MULT (default 4) workgroups per CU (conv3d_v4.hip)
    mult = int(os.environ.get("CWDM_V4_GRID_MULT", "4"))
    nblk = min(nblk, mult * torch.cuda.get_device_properties(0).multi_processor_count)
    buf = torch.zeros(nblk * 24, dtype=torch.int64, device="cuda")
    conv_bench.run_case(case, spec, 3, 1)  # warm
    lib().cwdm_debug_conv_stamps(ctypes.c_void_p(buf.data_ptr()))
    conv_bench.run_case(case, spec, 1, 1)
    torch.cuda.synchronize()
    lib().cwdm_debug_conv_stamps(None)
    st = buf.view(nblk, 24).cpu().tolist()
    nch = (spec[1] + spec[2]) // 16
    names = ["prologue (tile 0)"] + [f"chunk {c} (tile 0)" for c in range(min(nch, 8))]
    idx = [(0, 1)] + [((1 if c == 0 else 3 + c), 4 + c) for c in range(min(nch, 8))]
    names += ["epilogue (tile 0)", "rest of the tiles", "total"]
    idx += [(12, 13), (13, 15), (0, 15)]
    mean = lambda v: sum(v) / max(len(v), 1)
    print(f"{case}: {nblk} workgroups, {nch} chunks; cycles (mean / min / max)")
    for nm, (a, b) in zip(names, idx):
        v = [r[b] - r[a] for r in st]
        print(f"  {nm:20s} {mean(v):9.0f} {min(v):9d} {max(v):9d}")
    clk = [(r[15] - r[0]) / max(r[21] - r[20], 1) * 0.1 for r in st]
    print(f"  shader clock (s_memtime / s_memrealtime): mean {mean(clk):.2f} GHz, min {min(clk):.2f}, max {max(clk):.2f}")
    # co-residency: workgroups on the same (xcc, se/sh/cu)
    cu = collections.defaultdict(list)
    for i, r in enumerate(st):
        cu[(r[23] & 0xF, (r[22] >> 8) & 0xFF)].append((r[0], r[15], i))
    counts = collections.Counter(len(v) for v in cu.values())
    print(f"  CUs seen {len(cu)}; workgroups per CU histogram {dict(sorted(counts.items()))}")
    # max concurrency per CU and overlap fraction
    conc = []
    for v in cu.values():
        ev = sorted([(a, 1) for a, _, _ in v] + [(b, -1) for _, b, _ in v])
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        conc.append(m)
    print(f"  max concurrent workgroups per CU histogram {dict(sorted(collections.Counter(conc).items()))}")
    # phase offset between concurrent pairs: start-time difference relative to duration
    offs = []
    for v in cu.values():
        v.sort()
        for (a0, b0, _), (a1, b1, _) in zip(v, v[1:]):
            if a1 < b0:
                offs.append((a1 - a0) / max(b0 - a0, 1))
    if offs:
        offs.sort()
        print(f"  start offset of overlapping neighbours / duration: median {offs[len(offs) // 2]:.2f}, "
              f"p10 {offs[len(offs) // 10]:.2f}, p90 {offs[9 * len(offs) // 10]:.2f}")


if __name__ == "__main__":
    main()
