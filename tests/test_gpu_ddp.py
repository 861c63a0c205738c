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


def _model(P):
    from guided_diffusion import script_util
    args = script_util.run_sh_model_args(num_channels=32, channel_mult="1,2", num_res_blocks=1, num_groups=8)
    keys = script_util.model_and_diffusion_defaults().keys()
    model, diffusion = script_util.create_model_and_diffusion(**{k: args[k] for k in keys})
    model.set_compute_dtype("fp32")
    model.load_state_dict(P)
    return model.to("cuda"), diffusion


def _inputs():
    vols = cases.data.brats_batch(32, seed=8, batch=2)
    t = torch.tensor([37, 811])
    noise = torch.randn(2, 1, 32, 32, 32, generator=torch.Generator().manual_seed(9))
    return vols, t, noise


def _grad(model, diffusion, vols, t, noise):
    terms, _, _ = diffusion.training_losses(model, {k: v.cuda() for k, v in vols.items()}, t.cuda(), mode="i2i",
                                            contr="t1n", noise=noise.cuda())
    loss = terms["mse_wav"].mean()
    loss.backward()
    torch.cuda.synchronize()
    return model.flat_grad().detach().cpu().clone(), float(loss)


def _rank(rank, world, port, q):
    _setup()
    import torch.distributed as dist
    from cwdm_hip.ddp import GradBucketReducer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        model, diffusion = _model(ou.random_params(seed=41, **cases.C1_CFG))
        model._grad_hook = GradBucketReducer(bucket_bytes=256 << 10)   # several buckets for the small model
        vols, t, noise = _inputs()
        sl = slice(rank, rank + 1)
        g, loss = _grad(model, diffusion, {k: v[sl] for k, v in vols.items()}, t[sl], noise[sl])
        q.put((rank, g, loss))
    finally:
        dist.destroy_process_group()


def test_ddp_world2_batch1_equals_single_batch2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, g, loss = q.get(timeout=240)
        res[r] = (g, loss)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _setup()
    model, diffusion = _model(ou.random_params(seed=41, **cases.C1_CFG))
    vols, t, noise = _inputs()
    g_ref, loss_ref = _grad(model, diffusion, vols, t, noise)
    # both ranks hold the same averaged gradient, equal to the batch-2 gradient
    assert torch.equal(res[0][0], res[1][0])
    err = float((res[0][0].double() - g_ref.double()).norm() / g_ref.double().norm())
    assert err < 1e-5, err
    assert abs((res[0][1] + res[1][1]) / 2 - loss_ref) / loss_ref < 1e-5
