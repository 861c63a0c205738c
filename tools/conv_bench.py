"""Micro-benchmark of single conv3d launches (libcwdm C ABI) at U-Net shapes.

usage: python tools/conv_bench.py [--iters N] [--only NAME]
Prints one line per case: time per launch and TFLOP/s (algorithmic 2*MAC).
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-cwdm_amd"))

import torch  # noqa: E402

from cwdm_hip import _lib  # noqa: E402
from cwdm_hip._lib import check, lib  # noqa: E402

CASES = {
    # name: (grid, cin_a, cin_a1, cout, amode, gn, cin_b, rmode)
    "L0_64_64_gn": (128, 64, 0, 64, 0, True, 0, -1),
    "L0_64_64_gn_res": (128, 64, 0, 64, 0, True, 0, 0),
    "L0_64_64_gn_skip192": (128, 64, 0, 64, 0, True, 192, -1),
    "L0_128_128_up": (128, 128, 0, 128, 1, True, 0, -1),
    "L0_128_128_gn": (128, 128, 0, 128, 0, True, 0, -1),
    "L0_192_64_cat": (128, 128, 64, 64, 0, True, 0, -1),
    "L0_64_8_out": (128, 64, 0, 8, 0, True, 0, -1),
    "L0_64_8_out_nogn": (128, 64, 0, 8, 0, False, 0, -1),
    "L1_256_128_cat": (64, 128, 128, 128, 0, True, 0, -1),
    "L0_64_64_nogn": (128, 64, 0, 64, 0, False, 0, -1),
    "L0_192_64_cat_nogn": (128, 128, 64, 64, 0, False, 0, -1),
    "L1_128_128_gn": (64, 128, 0, 128, 0, True, 0, -1),
    "L1_128_128_nogn": (64, 128, 0, 128, 0, False, 0, -1),
    "L1_64_64_nogn": (64, 64, 0, 64, 0, False, 0, -1),
    "L0_128_64_nogn": (128, 128, 0, 64, 0, False, 0, -1),
    "L2_128_128_gn": (32, 128, 0, 128, 0, True, 0, -1),
    "L3_256_256_gn": (16, 256, 0, 256, 0, True, 0, -1),
    "L3_256_256_res": (16, 256, 0, 256, 0, False, 0, 0),
    "L4_256_256_gn": (8, 256, 0, 256, 0, True, 0, -1),
    "L4_256_256_nogn": (8, 256, 0, 256, 0, False, 0, -1),
    # config 5 (224^3 input -> 56^3 / 28^3 / 14^3 levels)
    "C5_L1_128_128_gn": (28, 128, 0, 128, 0, True, 0, -1),
    "C5_L1_64_128_gn": (28, 64, 0, 128, 0, True, 0, -1),
    "C5_L1_256_128_cat": (28, 128, 128, 128, 0, True, 0, -1),
    "C5_L2_128_128_gn": (14, 128, 0, 128, 0, True, 0, -1),
    "C5_L0_64_64_gn": (56, 64, 0, 64, 0, True, 0, -1),
    "C5_L0_64_64_nogn": (56, 64, 0, 64, 0, False, 0, -1),
    "C5_L0_128_64_cat_nogn": (56, 64, 64, 64, 0, False, 0, -1),
    # the down block's convs at 28^3 (64 -> 64 on the pooled input; conv2 adds the pooled x)
    "C5_D1_64_64_nogn": (28, 64, 0, 64, 0, False, 0, -1),
    "C5_D1_64_64_res": (28, 64, 0, 64, 0, False, 0, 0),
}


def run_case(name, spec, iters, dtype):
    n, ca0, ca1, cout, amode, gn, cb, rmode = spec
    dev = "cuda"
    tdt = torch.bfloat16 if dtype == _lib.CWDM_BF16 else torch.float32
    L = lib()
    src_n = n // 2 if amode == 1 else n
    a0 = torch.randn(1, src_n, src_n, src_n, ca0, device=dev).to(tdt)
    a1 = torch.randn(1, src_n, src_n, src_n, ca1, device=dev).to(tdt) if ca1 else None
    cin = ca0 + ca1
    w = torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.02
    pw = torch.empty(L.cwdm_conv3d_packed_bytes(cout, cin, 3, dtype), dtype=torch.uint8, device=dev)
    check(L.cwdm_conv3d_pack(ctypes.c_void_p(w.data_ptr()), cout, cin, 3, dtype, ctypes.c_void_p(pw.data_ptr()), None))
    pb = None
    if cb:
        wb = torch.randn(cout, cb, 1, 1, 1, device=dev) * 0.02
        pb = torch.empty(L.cwdm_conv3d_packed_bytes(cout, cb, 1, dtype), dtype=torch.uint8, device=dev)
        check(L.cwdm_conv3d_pack(ctypes.c_void_p(wb.data_ptr()), cout, cb, 1, dtype, ctypes.c_void_p(pb.data_ptr()),
                                 None))
        b0 = torch.randn(1, n, n, n, cb, device=dev).to(tdt)
    gnb = torch.stack([torch.ones(1, cin, device=dev), torch.zeros(1, cin, device=dev)], -1).contiguous()
    bias = torch.zeros(cout, device=dev)
    res = torch.randn(1, n, n, n, cout, device=dev).to(tdt) if rmode >= 0 else None
    out = torch.empty(1, n, n, n, cout, device=dev, dtype=torch.float32 if cout == 8 else tdt)
    parts = L.cwdm_conv3d_parts(dtype, n, n, n, cout)
    st = torch.empty(1, parts, cout, 2, device=dev)
    d = _lib.ConvDesc()
    d.dtype, d.B, d.D, d.H, d.W, d.cout = dtype, 1, n, n, n, cout
    d.a0, d.a_c0 = a0.data_ptr(), ca0
    d.a1, d.a_c1 = (a1.data_ptr(), ca1) if a1 is not None else (None, 0)
    d.a_mode = amode
    d.a_gn = gnb.data_ptr() if gn else None
    d.a_w = pw.data_ptr()
    if cb:
        d.b0, d.b_c0, d.b_w = b0.data_ptr(), cb, pb.data_ptr()
    d.bias, d.bias_bstride = bias.data_ptr(), 0
    d.res, d.res_mode = (res.data_ptr() if res is not None else None), rmode
    d.out, d.out_dtype = out.data_ptr(), (_lib.CWDM_F32 if cout == 8 else dtype)
    d.stats = st.data_ptr() if cout != 8 else None
    nws = L.cwdm_conv3d_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=dev)
    d.workspace, d.ws_bytes = ws.data_ptr(), nws
    for _ in range(3):
        check(L.cwdm_conv3d_forward(ctypes.byref(d), None))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        check(L.cwdm_conv3d_forward(ctypes.byref(d), None))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2.0 * n ** 3 * cout * (27 * cin + cb)
    print(f"{name:24s} {ms * 1e3:9.1f} us  {flops / ms / 1e9:8.1f} TFLOP/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    dt = _lib.CWDM_BF16 if args.dtype == "bf16" else _lib.CWDM_F32
    for name, spec in CASES.items():
        if args.only and not any(o == name for o in args.only.split(",")) and args.only not in name:
            continue
        run_case(name, spec, args.iters, dt)


if __name__ == "__main__":
    main()
