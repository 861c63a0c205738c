"""Distributed helpers (API of guided_diffusion/dist_util.py:20-107).

One process per GPU.  Under ``torchrun`` (RANK/WORLD_SIZE/LOCAL_RANK in the
environment) ``setup_dist`` joins that job -- backend "nccl" (= RCCL over xGMI
on ROCm) when a GPU is visible, "gloo" otherwise -- and binds the process to
GPU LOCAL_RANK.  Without it, a single-process group is created on 127.0.0.1,
as the reference does (it hard-codes WORLD_SIZE=1, :41-46).  ``sync_params``
broadcasts rank 0's weights (a no-op in the reference, :93-99, which therefore
never averaged gradients across ranks; TrainLoop here does, see train_util).
"""
import io
import os
import socket

import torch as th
import torch.distributed as dist

GPUS_PER_NODE = 8
SETUP_RETRY_COUNT = 3


def _find_free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
    finally:
        s.close()


def setup_dist(devices=(0,)):
    if dist.is_initialized():
        return
    launched = "RANK" in os.environ and "WORLD_SIZE" in os.environ
    if not launched:
        os.environ["RANK"] = "0"
        os.environ["WORLD_SIZE"] = "1"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(_find_free_port())
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    cuda = th.cuda.device_count() > 0 and th.cuda.is_available()
    backend = "nccl" if cuda else "gloo"
    kw = {}
    if cuda:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if launched:
            idx = local % th.cuda.device_count()
        else:
            first = devices[0] if isinstance(devices, (list, tuple)) else devices
            idx = int(first) % th.cuda.device_count()
        th.cuda.set_device(idx)
        # bind the communicator to this rank's GPU up front (no "guessing device
        # ID based on global rank" at the first collective)
        kw["device_id"] = th.device("cuda", idx)
    dist.init_process_group(backend=backend, init_method="env://", **kw)


def dev(device_number=None):
    """The device of this rank (reference :54-71; cuda:LOCAL_RANK under torchrun)."""
    if isinstance(device_number, (list, tuple)):
        return [dev(k) for k in device_number]
    if th.cuda.is_available():
        n = th.cuda.device_count()
        if device_number is None:
            device_number = int(os.environ.get("LOCAL_RANK", th.cuda.current_device()))
        if n == 1:
            return th.device("cuda")
        if device_number < n:
            return th.device(f"cuda:{device_number}")
        raise ValueError(f"requested device number {device_number} (0-indexed) but only {n} devices available")
    return th.device("cpu")


def load_state_dict(path, **kwargs):
    """Reference :74-90.  Loads tensors only (weights_only=True)."""
    with open(path, "rb") as f:
        data = f.read()
    kwargs.setdefault("weights_only", True)
    return th.load(io.BytesIO(data), **kwargs)


def sync_params(params):
    """Broadcast rank 0's parameters to every rank (in place; each parameter's
    version counter is bumped so caches keyed on it -- the native UNetModel's
    packed weights -- see the new values)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    with th.no_grad():
        for p in params:
            dist.broadcast(p.data, 0)
            th.autograd.graph.increment_version(p)
