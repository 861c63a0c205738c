"""Phase stamps of the output head as it runs inside the sampling step (the
fused sampler epilogue, head2_kernel SAMP): one eager bench.py step with the
stamps library; the head is the step's last kernel, so the shared stamps buffer
holds its phases afterwards.

usage: CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 python tools/head_step_stamps.py"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import bench  # noqa: E402
import head_stamps  # noqa: E402
from cwdm_hip._lib import lib  # noqa: E402


def main():
    args = argparse.Namespace(grid=128, dtype="bf16")
    device = torch.device("cuda", 0)
    model, diffusion = bench.build(args, device)
    n = args.grid
    from cwdm_hip import ops
    cond = torch.empty(1, 24, n, n, n, device=device)
    V = n ** 3
    for k in range(3):
        vol = bench.phantom_gpu(2 * n, 100 + k, device)
        ops.dwt3d(vol, lll_div3=True, out=cond[:, 8 * k:], out_strides=(V, 24 * V, 0, 1))
    x_T = torch.randn(1, 8, n, n, n, device=device)
    T = diffusion.num_timesteps
    loop = diffusion._native_loop(model, x_T, list(range(T))[::-1][:4], cond, True, graph=False)
    next(loop)
    torch.cuda.synchronize()
    nwg = torch.cuda.get_device_properties(0).multi_processor_count
    buf = torch.zeros(nwg * 64, dtype=torch.int64, device="cuda")
    lib().cwdm_debug_conv_stamps(ctypes.c_void_p(buf.data_ptr()))
    next(loop)
    torch.cuda.synchronize()
    lib().cwdm_debug_conv_stamps(None)
    loop.close()
    head_stamps.report("in-step head (SAMP)", buf, nwg)


if __name__ == "__main__":
    main()
