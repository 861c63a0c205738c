"""Time cwdm_conv3d_wgrad on production shapes (128^3 grid, bf16), with and
without the GroupNorm+SiLU prologue, to locate the kernel's bound.
usage: python tools/wgrad_bench.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-cwdm_amd"))

import torch  # noqa: E402

from cwdm_hip import _lib  # noqa: E402
from cwdm_hip._lib import check, lib  # noqa: E402


def run(n, cin, cout, gn, iters=5, cm=False, umode=0):
    dev = "cuda"
    sn = n // 2 if umode else n
    if cm:   # the training forward's kept activation: chunk-major [cin/16][V][16]
        x = torch.randn(1, cin // 16, sn, sn, sn, 16, device=dev).to(torch.bfloat16)
    else:
        x = torch.randn(1, sn, sn, sn, cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(1, n, n, n, cout, device=dev).to(torch.bfloat16)
    g = torch.stack([1 + 0.1 * torch.randn(1, cin), 0.1 * torch.randn(1, cin)], -1).contiguous().to(dev)
    dw = torch.zeros(cout, cin, 3, 3, 3, device=dev)
    ws = torch.empty(lib().cwdm_conv3d_wgrad_workspace_bytes(cout, cin, 3), dtype=torch.uint8, device=dev)
    d = _lib.WgradDesc()
    d.dtype, d.B, d.D, d.H, d.W, d.ksize = _lib.CWDM_BF16, 1, n, n, n, 3
    d.u0, d.u_c0, d.u1, d.u_c1, d.u_mode = x.data_ptr(), cin, None, 0, umode
    d.u_gn = g.data_ptr() if (gn and not cm) else None
    d.u_cm = 1 if cm else 0
    d.dy, d.dy_cs, d.cout, d.dw, d.workspace = dy.data_ptr(), cout, cout, dw.data_ptr(), ws.data_ptr()
    d.ws_bytes = ws.numel()
    for _ in range(2):
        check(lib().cwdm_conv3d_wgrad(ctypes.byref(d), None))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        check(lib().cwdm_conv3d_wgrad(ctypes.byref(d), None))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    fl = 2.0 * n ** 3 * cin * cout * 27
    tag = "dma" if cm else ("gn" if gn else "plain")
    print(f"wgrad n={n} cin={cin} cout={cout} {tag} up={umode}: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s",
          flush=True)


if __name__ == "__main__":
    if "--dma" in sys.argv:   # the kept-activation (LDS-DMA) kernel on the R0 / R1 training shapes
        cases = ((128, 64, 64, 0), (128, 192, 64, 0), (128, 128, 64, 0), (128, 128, 128, 1),
                 (64, 128, 128, 0), (64, 256, 128, 0), (64, 384, 128, 0))
        if "--case" in sys.argv:   # one of them (index), e.g. for a PMC pass
            cases = (cases[int(sys.argv[sys.argv.index("--case") + 1])],)
        for n, cin, cout, um in cases:
            run(n, cin, cout, False, cm=True, umode=um)
        sys.exit(0)
    for n, cin, cout in ((128, 64, 64), (128, 128, 64), (64, 128, 128), (32, 256, 256)):
        for gn in (True, False):
            run(n, cin, cout, gn)
