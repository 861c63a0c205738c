"""Utility surface of guided_diffusion/nn.py (reference :1-170).

These helpers keep the reference names for callers that import them
(scripts, losses).  The U-Net itself does not use them: GroupNorm32+SiLU,
Conv3d, pooling/upsampling and the timestep embedding are fused into the
libcwdm kernels behind ``unet.UNetModel``.
"""
import math

import torch as th
import torch.nn as nn


class SiLU(nn.Module):
    def forward(self, x):
        return x * th.sigmoid(x)


class GroupNorm32(nn.GroupNorm):
    def forward(self, x):
        return super().forward(x.float()).type(x.dtype)


def conv_nd(dims, *args, **kwargs):
    if dims == 1:
        return nn.Conv1d(*args, **kwargs)
    if dims == 2:
        return nn.Conv2d(*args, **kwargs)
    if dims == 3:
        return nn.Conv3d(*args, **kwargs)
    raise ValueError(f"unsupported dimensions: {dims}")


def linear(*args, **kwargs):
    return nn.Linear(*args, **kwargs)


def avg_pool_nd(dims, *args, **kwargs):
    if dims == 1:
        return nn.AvgPool1d(*args, **kwargs)
    if dims == 2:
        return nn.AvgPool2d(*args, **kwargs)
    if dims == 3:
        return nn.AvgPool3d(*args, **kwargs)
    raise ValueError(f"unsupported dimensions: {dims}")


def update_ema(target_params, source_params, rate=0.99):
    for targ, src in zip(target_params, source_params):
        targ.detach().mul_(rate).add_(src, alpha=1 - rate)


def zero_module(module):
    for p in module.parameters():
        p.detach().zero_()
    return module


def scale_module(module, scale):
    for p in module.parameters():
        p.detach().mul_(scale)
    return module


def mean_flat(tensor):
    """Mean over all dims from 2 on (reference nn.py:86-90).  A large row is
    reduced as 256 equal slices then their mean: ROCm torch runs one 64-thread
    workgroup per output row (the training loss's [1, 8, 128^3] took 296 us,
    one per output channel)."""
    n = 1
    for s in tensor.shape[2:]:
        n *= s
    if tensor.is_cuda and tensor.dim() > 2 and n >= (1 << 16) and n % 256 == 0:
        return tensor.reshape(*tensor.shape[:2], 256, n // 256).mean(-1).mean(-1)
    return tensor.mean(dim=list(range(2, len(tensor.shape))))


def normalization(channels, groups=32):
    return GroupNorm32(groups, channels)


def timestep_embedding(timesteps, dim, max_period=10000):
    """Sinusoidal embedding, cos first (reference nn.py:103-121)."""
    half = dim // 2
    freqs = th.exp(-math.log(max_period) * th.arange(start=0, end=half, dtype=th.float32) / half).to(
        device=timesteps.device)
    args = timesteps[:, None].float() * freqs[None]
    embedding = th.cat([th.cos(args), th.sin(args)], dim=-1)
    if dim % 2:
        embedding = th.cat([embedding, th.zeros_like(embedding[:, :1])], dim=-1)
    return embedding


def checkpoint(func, inputs, params, flag):
    """Activation checkpointing is not needed on MI355X (288 GB HBM holds the
    128^3 activation set many times over); the flag is accepted and ignored."""
    return func(*inputs)
