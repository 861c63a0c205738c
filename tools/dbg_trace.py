"""Debug helper: production U-Net block trace (bf16/fp16, a conv path policy) vs
the oracle's fp32 trace; prints the first blocks that go wrong.
usage: python tools/dbg_trace.py D H W [dtype] [path]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fast-cwdm_amd"))
import torch  # noqa: E402

from oracle import unet as ou  # noqa: E402


def main():
    D, H, W = (int(a) for a in sys.argv[1:4])
    dtype = sys.argv[4] if len(sys.argv) > 4 else "bf16"
    path = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    from cwdm_hip._lib import lib
    from guided_diffusion.unet import UNetModel
    cfg = dict(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2, channel_mult=(1, 2, 2, 4, 4))
    P = ou.random_params(seed=13)
    lib().cwdm_conv3d_set_path(path)
    m = UNetModel(image_size=32, in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2,
                  attention_resolutions=(), channel_mult=cfg["channel_mult"], dims=3, resblock_updown=True,
                  bottleneck_attention=False, resample_2d=False, num_groups=32, compute_dtype=dtype)
    m.load_state_dict(P)
    m = m.to("cuda")
    g = torch.Generator().manual_seed(8)
    x = torch.randn(1, 32, D, H, W, generator=g)
    t = torch.tensor([700])
    trace = []
    ref = ou.unet_forward(P, x, t, trace=trace)
    with torch.no_grad():
        out = m(x.to("cuda"), t.to("cuda"))
    torch.cuda.synchronize()
    ws = m.plan.workspace(1, D, H, W, "cuda")
    got = m.plan.trace_tensors(ws, 1, D, H, W)
    for i, (gt, rf) in enumerate(zip(got, trace)):
        if gt is None:
            continue
        a = gt.float().permute(0, 4, 1, 2, 3).cpu()
        err = float((a - rf).abs().max() / rf.abs().max())
        nan = int(torch.isnan(a).sum())
        print(f"block {i:2d} shape {tuple(a.shape)} rel {err:.3e} nan {nan}", flush=True)
    o = out.cpu()
    print("out rel", float((o - ref).abs().max() / ref.abs().max()), "nan", int(torch.isnan(o).sum()))




def where_bad():
    """python tools/dbg_trace.py where D H W: positions of the wrong conv_in outputs."""
    D, H, W = (int(a) for a in sys.argv[2:5])
    from guided_diffusion.unet import UNetModel
    from cwdm_hip._lib import lib
    lib().cwdm_conv3d_set_path(2)
    P = ou.random_params(seed=13)
    m = UNetModel(image_size=32, in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2,
                  attention_resolutions=(), channel_mult=(1, 2, 2, 4, 4), dims=3, resblock_updown=True,
                  bottleneck_attention=False, resample_2d=False, num_groups=32, compute_dtype="bf16")
    m.load_state_dict(P)
    m = m.to("cuda")
    g = torch.Generator().manual_seed(8)
    x = torch.randn(1, 32, D, H, W, generator=g)
    trace = []
    ou.unet_forward(P, x, torch.tensor([700]), trace=trace)
    with torch.no_grad():
        m(x.to("cuda"), torch.tensor([700]).to("cuda"))
    torch.cuda.synchronize()
    got = m.plan.trace_tensors(m.plan.workspace(1, D, H, W, "cuda"), 1, D, H, W)[0].float().cpu()[0]  # D H W C
    ref = trace[0][0].permute(1, 2, 3, 0)
    bad = (got - ref).abs() > 0.05 * ref.abs().max()
    print("bad", int(bad.sum()), "of", bad.numel())
    idx = bad.nonzero()
    print("z", sorted(set(idx[:, 0].tolist()))[:40])
    print("y", sorted(set(idx[:, 1].tolist()))[:40])
    print("x", sorted(set(idx[:, 2].tolist()))[:40])
    print("c", sorted(set(idx[:, 3].tolist()))[:70])
    for k in range(min(12, len(idx))):
        z, y, xx, c = idx[k].tolist()
        print(z, y, xx, c, float(got[z, y, xx, c]), float(ref[z, y, xx, c]))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "where":
    where_bad()
    sys.exit(0)



def standalone():
    """python tools/dbg_trace.py alone D H W: conv_in-like conv via cwdm_conv3d_forward, v5 vs v4, repeated."""
    import ctypes
    import math
    D, H, W = (int(a) for a in sys.argv[2:5])
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    L = lib()
    g = torch.Generator().manual_seed(8)
    B, cin, cout = 1, 32, 64
    x = torch.randn(B, D, H, W, cin, generator=g).to("cuda", torch.bfloat16)
    w = (torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)).to("cuda")
    bias = (torch.randn(cout, generator=g) * 0.1).to("cuda")
    nb = L.cwdm_conv3d_packed_bytes(cout, cin, 3, _lib.CWDM_BF16)
    pk = torch.empty(nb, dtype=torch.uint8, device="cuda")
    check(L.cwdm_conv3d_pack(ctypes.c_void_p(w.data_ptr()), cout, cin, 3, _lib.CWDM_BF16,
                             ctypes.c_void_p(pk.data_ptr()), None))
    parts = L.cwdm_conv3d_parts(_lib.CWDM_BF16, D, H, W, cout)
    res = {}
    for path in (3, 2, 2, 3, 2):
        L.cwdm_conv3d_set_path(path)
        out = torch.full((B, D, H, W, cout), float("nan"), device="cuda", dtype=torch.bfloat16)
        st = torch.zeros(B, parts, cout, 2, device="cuda")
        d = _lib.ConvDesc()
        d.dtype, d.B, d.D, d.H, d.W, d.cout = _lib.CWDM_BF16, B, D, H, W, cout
        d.a0, d.a_c0, d.a_w = x.data_ptr(), cin, pk.data_ptr()
        d.bias, d.res_mode = bias.data_ptr(), -1
        d.out, d.out_dtype, d.stats = out.data_ptr(), _lib.CWDM_BF16, st.data_ptr()
        nws = L.cwdm_conv3d_workspace_bytes(ctypes.byref(d))
        ws = torch.empty(max(nws, 1), dtype=torch.uint8, device="cuda")
        d.workspace, d.ws_bytes = ws.data_ptr(), nws
        check(L.cwdm_conv3d_forward(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        if path == 3:
            res["v4"] = out.float().cpu()
        else:
            o = out.float().cpu()
            bad = int(((o - res["v4"]).abs() > 1e-2).sum())
            print("v5 run: bad", bad, "nan", int(torch.isnan(o).sum()), flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "alone":
    standalone()
    sys.exit(0)


if __name__ == "__main__" and sys.argv[1] not in ("where", "alone"):
    main()
