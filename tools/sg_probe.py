"""Probe of the small-grid conv kernel (conv3d_sg.hip) with single-tap identity
weights: for each tap, out[co] should be the input channel co shifted by the
tap.  Prints the max error per tap and per (tap, output channel group)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-cwdm_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from cwdm_hip import _lib  # noqa: E402
from cwdm_hip._lib import check, lib  # noqa: E402

L = lib()
D, H, W = 4, 4, 16
cin, cout = 32, 64
dev = "cuda"
x = torch.randn(1, cin, D, H, W)
for tap in range(27):
    kz, ky, kx = tap // 9, (tap // 3) % 3, tap % 3
    w = torch.zeros(cout, cin, 3, 3, 3)
    for co in range(cout):
        w[co, co % cin, kz, ky, kx] = 1.0 + co * 0.001
    ref = F.conv3d(x.to(torch.bfloat16).float(), w.to(torch.bfloat16).float(), padding=1)
    a0 = x.permute(0, 2, 3, 4, 1).contiguous().to(dev, torch.bfloat16)
    pw = torch.empty(L.cwdm_conv3d_packed_bytes(cout, cin, 3, _lib.CWDM_BF16), dtype=torch.uint8, device=dev)
    check(L.cwdm_conv3d_pack(ctypes.c_void_p(w.to(dev).data_ptr()), cout, cin, 3, _lib.CWDM_BF16,
                             ctypes.c_void_p(pw.data_ptr()), None))
    out = torch.empty(1, D, H, W, cout, device=dev, dtype=torch.bfloat16)
    bias = torch.zeros(cout, device=dev)
    d = _lib.ConvDesc()
    d.dtype, d.B, d.D, d.H, d.W, d.cout = _lib.CWDM_BF16, 1, D, H, W, cout
    d.a0, d.a_c0 = a0.data_ptr(), cin
    d.a1, d.a_c1 = None, 0
    d.a_mode = 0
    d.a_gn = None
    d.a_w = pw.data_ptr()
    d.bias, d.bias_bstride = bias.data_ptr(), 0
    d.res, d.res_mode = None, -1
    d.out, d.out_dtype = out.data_ptr(), _lib.CWDM_BF16
    d.stats = None
    nws = L.cwdm_conv3d_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=dev)
    d.workspace, d.ws_bytes = ws.data_ptr(), nws
    check(L.cwdm_conv3d_forward(ctypes.byref(d), None))
    torch.cuda.synchronize()
    got = out.float().cpu().permute(0, 4, 1, 2, 3)
    err = (got - ref).abs()
    per_cg = [float(err[:, 16 * g:16 * g + 16].max()) for g in range(4)]
    # where is the first wrong value, and which input does it look like
    bad = (err > 0.05).nonzero()
    msg = ""
    if len(bad):
        _, co, z, y, xx = bad[0].tolist()
        v = float(got[0, co, z, y, xx])
        hits = (x.to(torch.bfloat16).float()[0] - v / (1.0 + co * 0.001)).abs() < 1e-2
        where = hits.nonzero()[:3].tolist()
        msg = f" first bad co={co} z={z} y={y} x={xx} got={v:.3f} ref={float(ref[0, co, z, y, xx]):.3f} matches input at {where}"
    print(f"tap {tap:2d} (kz,ky,kx)=({kz},{ky},{kx}) max err {float(err.max()):.3f} per 16-ch group {['%.2f' % e for e in per_cg]}{msg}", flush=True)
