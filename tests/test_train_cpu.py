"""CPU tests of the training host logic: the data-parallel gradient reducer
over gloo (world_size 2, the N>1 path of config 3 without a GPU), timestep
samplers, checkpoint-name parsing and the logger."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reducer_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fast-cwdm_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cwdm_hip.ddp import GradBucketReducer, broadcast_params
        N = 100
        flat = torch.arange(N, dtype=torch.float32) * (rank + 1)
        red = GradBucketReducer(bucket_bytes=25 * 4)
        # segment order of the native backward: descending adjacent ranges, plus a gap
        for seg, (off, n) in enumerate([(90, 10), (70, 20), (50, 20), (10, 30), (0, 10)]):
            red(seg, flat, off, n)
        red(None, flat, 0, N)
        # the range [40, 50) was never reported: only the final 1/world scaling touches it
        exp = torch.arange(N, dtype=torch.float32) * (1 + world) / 2
        exp[40:50] = torch.arange(40, 50, dtype=torch.float32) * (rank + 1) / world
        ok = torch.allclose(flat, exp)
        p = [torch.full((3,), float(rank)), torch.full((2, 2), float(rank) + 10)]
        broadcast_params(p)
        ok = ok and float(p[0][0]) == 0.0 and float(p[1][0, 0]) == 10.0
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_grad_bucket_reducer_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_reducer_single_process_is_noop():
    from cwdm_hip.ddp import GradBucketReducer
    flat = torch.arange(10.0)
    r = GradBucketReducer()
    r(0, flat, 5, 5)
    r(None, flat, 0, 10)
    assert torch.equal(flat, torch.arange(10.0))


class _Diff:
    num_timesteps = 50


def test_uniform_sampler_matches_numpy_stream():
    from guided_diffusion.resample import UniformSampler, create_named_schedule_sampler
    s = create_named_schedule_sampler("uniform", _Diff(), 50)
    assert isinstance(s, UniformSampler)
    np.random.seed(3)
    t, w = s.sample(6, "cpu")
    np.random.seed(3)
    ref = np.random.choice(50, size=(6,), p=np.ones(50) / 50)
    assert t.tolist() == ref.tolist() and torch.all(w == 1)
    assert UniformSampler(_Diff()).weights().shape == (50,)


def test_loss_second_moment_sampler():
    from guided_diffusion.resample import LossSecondMomentResampler
    s = LossSecondMomentResampler(_Diff(), history_per_term=2)
    assert np.all(s.weights() == 1)
    for _ in range(2):
        s.update_with_all_losses(list(range(50)), [float(k + 1) for k in range(50)])
    w = s.weights()
    assert abs(w.sum() - 1) < 1e-9 and w[49] > w[0]


def test_parse_resume_step_and_logger(tmp_path, capsys):
    from guided_diffusion import logger
    from guided_diffusion.train_util import parse_resume_step_from_filename
    assert parse_resume_step_from_filename("/x/brats_t1n_012000.pt") == 12000
    assert parse_resume_step_from_filename("/x/model_BEST.pt") == 0
    logger.configure(str(tmp_path), ["stdout", "csv"])
    logger.logkv("step", 1)
    logger.logkv_mean("loss", 1.0)
    logger.logkv_mean("loss", 3.0)
    d = logger.dumpkvs()
    assert d["loss"] == 2.0
    assert os.path.exists(os.path.join(tmp_path, "progress.csv"))
    logger.configure(None, ["stdout"])


def test_setup_dist_single_process_gloo():
    from guided_diffusion import dist_util
    if dist.is_initialized():
        pytest.skip("process group already initialised")
    env = {k: os.environ.get(k) for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    try:
        dist_util.setup_dist()
        assert dist.get_world_size() == 1
        assert dist_util.dev() == torch.device("cpu")
    finally:
        dist.destroy_process_group()
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
