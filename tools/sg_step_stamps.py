"""In-step phase stamps of the small-grid conv (csrc/conv3d_sg.hip): one eager
production forward at 128^3 (bf16) with the stamps buffer set, so the buffer
holds the LAST small-grid launch of the step (a 16^3 decoder conv), cold caches
and all, as the step runs it.  Per workgroup: realtime start / end (100 MHz),
s_memtime phases.  needs the stamps build (tools/build_ab_lib.sh stamps HEAD
STAMPS=1; CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1).
usage: python tools/sg_step_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-cwdm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from cwdm_hip._lib import lib  # noqa: E402


def main():
    class A:
        dtype = "bf16"
    dev = torch.device("cuda", 0)
    model, diffusion = bench.build(A, dev)
    n = 128
    x = torch.randn(1, 32, n, n, n, device=dev)
    t = torch.tensor([500.0], device=dev)
    with torch.no_grad():
        model(x, t)
        torch.cuda.synchronize()
        buf = torch.zeros(4096 * 24, dtype=torch.int64, device=dev)
        lib().cwdm_debug_conv_stamps(ctypes.c_void_p(buf.data_ptr()))
        model(x, t)
        torch.cuda.synchronize()
        lib().cwdm_debug_conv_stamps(None)
    st = [r for r in buf.view(4096, 24).cpu().tolist() if r[20] != 0]
    # only the small-grid kernel writes slots 20 / 21 (realtime) in this layout; others may have
    # written other slots of low workgroups: keep the rows of the last sg launch (consistent 20/21)
    st = [r for r in st if r[21] > r[20]]
    print(f"{len(st)} workgroups")
    t0 = min(r[20] for r in st)
    starts = sorted((r[20] - t0) / 100.0 for r in st)
    ends = sorted((r[21] - t0) / 100.0 for r in st)
    life = sorted((r[21] - r[20]) / 100.0 for r in st)
    q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))]  # noqa: E731
    print(f"start us: min {starts[0]:.2f} p50 {q(starts, .5):.2f} p90 {q(starts, .9):.2f} max {starts[-1]:.2f}")
    print(f"end   us: min {ends[0]:.2f} p50 {q(ends, .5):.2f} p90 {q(ends, .9):.2f} max {ends[-1]:.2f}")
    print(f"life  us: min {life[0]:.2f} p50 {q(life, .5):.2f} p90 {q(life, .9):.2f} max {life[-1]:.2f}")
    mean = lambda v: sum(v) / max(len(v), 1)  # noqa: E731
    print(f"cycles: first DMA {mean([r[1] - r[0] for r in st]):.0f}, loop {mean([r[12] - r[1] for r in st]):.0f}, "
          f"epilogue {mean([r[15] - r[12] for r in st]):.0f}, total {mean([r[15] - r[0] for r in st]):.0f}")
    for c in range(8):
        v = [r[4 + c] - (r[1] if c == 0 else r[3 + c]) for r in st if r[4 + c]]
        if v:
            print(f"  chunk {c}: {mean(v):.0f} cycles")


if __name__ == "__main__":
    main()
