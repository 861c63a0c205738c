"""Data-parallel pin: two ranks x batch 1 with the bucketed
gradient all-reduce overlapped with the segmented native backward equal one
process x batch 2 (the loss is a batch mean, so the DDP average is exactly the
batch-2 gradient up to fp32 reduction order).  Both ranks share the one GPU of
the test box and talk over gloo; the production run uses RCCL with one GPU per
rank, the reducer code is the same."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import cases, unet as ou

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    import sys
    for p in (os.path.join(ROOT, "fast-cwdm_amd"), ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)


# "c1": the config-1 tiny U-Net on 32^3 images; "prod": the run.sh U-Net
# (81.5 M parameters) on 64^3 images, the DMA-staged conv kernel forced
# wherever the shape allows (forward and dgrad)
CASES = {"c1": dict(overrides=dict(num_channels=32, channel_mult="1,2", num_res_blocks=1, num_groups=8),
                    params=lambda: ou.random_params(seed=41, **cases.C1_CFG), size=32, path=0),
         "prod": dict(overrides={}, params=lambda: ou.random_params(seed=43), size=64, path=2)}


def _model(which):
    from guided_diffusion import script_util
    args = script_util.run_sh_model_args(**CASES[which]["overrides"])
    keys = script_util.model_and_diffusion_defaults().keys()
    model, diffusion = script_util.create_model_and_diffusion(**{k: args[k] for k in keys})
    model.set_compute_dtype("fp32")
    model.load_state_dict(CASES[which]["params"]())
    return model.to("cuda"), diffusion


def _inputs(which):
    n = CASES[which]["size"]
    vols = cases.data.brats_batch(n, seed=8, batch=2)
    t = torch.tensor([37, 811])
    noise = torch.randn(2, 1, n, n, n, generator=torch.Generator().manual_seed(9))
    return vols, t, noise


def _set_path(which):
    from cwdm_hip._lib import lib
    return lib().cwdm_conv3d_set_path(CASES[which]["path"])


def _grad(model, diffusion, vols, t, noise):
    terms, _, _ = diffusion.training_losses(model, {k: v.cuda() for k, v in vols.items()}, t.cuda(), mode="i2i",
                                            contr="t1n", noise=noise.cuda())
    loss = terms["mse_wav"].mean()
    loss.backward()
    torch.cuda.synchronize()
    return model.flat_grad().detach().cpu().clone(), float(loss.detach())


def _rank(rank, world, port, q, which, outdir):
    _setup()
    import torch.distributed as dist
    from cwdm_hip.ddp import GradBucketReducer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        _set_path(which)
        model, diffusion = _model(which)
        model._grad_hook = GradBucketReducer(bucket_bytes=(256 << 10) if which == "c1" else (16 << 20))
        vols, t, noise = _inputs(which)
        sl = slice(rank, rank + 1)
        g, loss = _grad(model, diffusion, {k: v[sl] for k, v in vols.items()}, t[sl], noise[sl])
        # through a file: a 326 MB tensor in the queue is shared memory that
        # dies with this process
        path = os.path.join(outdir, f"grad{rank}.pt")
        torch.save(g, path)
        q.put((rank, path, loss))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("which", ["c1", "prod"])
def test_ddp_world2_batch1_equals_single_batch2(which, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q, which, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, path, loss = q.get(timeout=240)
        res[r] = (torch.load(path, weights_only=True), loss)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _setup()
    prev = _set_path(which)
    try:
        model, diffusion = _model(which)
        vols, t, noise = _inputs(which)
        g_ref, loss_ref = _grad(model, diffusion, vols, t, noise)
    finally:
        from cwdm_hip._lib import lib
        lib().cwdm_conv3d_set_path(prev)
    # both ranks hold the same averaged gradient, equal to the batch-2 gradient
    assert torch.equal(res[0][0], res[1][0])
    err = float((res[0][0].double() - g_ref.double()).norm() / g_ref.double().norm())
    assert err < 1e-5, err
    assert abs((res[0][1] + res[1][1]) / 2 - loss_ref) / loss_ref < 1e-5


def _rccl_rank(port, q):
    """One rank on RCCL ("nccl" backend): the bucketed reducer's async
    all-reduces on the communicator stream, overlapped with the segmented
    backward and waited stream-ordered, must leave the gradient unchanged at
    world size 1 (sum over one rank, divided by one)."""
    _setup()
    import torch.distributed as dist
    from cwdm_hip.ddp import GradBucketReducer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        model, diffusion = _model("c1")
        vols, t, noise = _inputs("c1")
        g_plain, _ = _grad(model, diffusion, vols, t, noise)
        red = GradBucketReducer(bucket_bytes=256 << 10, force=True, timing=True)
        model._grad_hook = red
        for p in model.parameters():
            p.grad = None
        g_red, _ = _grad(model, diffusion, vols, t, noise)
        bwd_end, buckets = red.timeline()
        q.put((red.launched, float((g_red - g_plain).abs().max()), float(g_plain.abs().max()), bwd_end, buckets))
    finally:
        dist.destroy_process_group()


def test_reducer_over_rccl_world1():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank, args=(_free_port(), q))
    p.start()
    launched, diff, scale, bwd_end, buckets = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert launched >= 2          # several buckets went through RCCL
    assert diff <= 1e-6 * scale, (diff, scale)
    # overlap, measured on the GPU timeline: bucket collectives start (on the
    # reducer's stream) while later backward segments still run on the compute
    # stream, i.e. before the backward's last segment ends
    assert len(buckets) == launched
    early = [b for b in buckets if b[1] < bwd_end]
    print("backward end %.3f ms; buckets (ready, start, end) ms:" % bwd_end, buckets)
    assert len(early) >= launched - 1, (bwd_end, buckets)
    assert all(s >= r - 1e-3 for r, s, _ in buckets)   # a collective never starts before its gradients
