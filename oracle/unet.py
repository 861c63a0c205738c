"""Oracle: functional 3D U-Net denoiser (TEST INFRASTRUCTURE ONLY).

A functional restatement of the reference ``UNetModel`` as configured by
run.sh (no attention, resblock_updown=True, use_scale_shift_norm=False,
additive_skips=False, resample_2d=False): topology from
guided_diffusion/unet.py:482-725, ResBlock._forward :285-311,
Up/Downsample :40-100, forward :754-800; primitives from
guided_diffusion/nn.py (GroupNorm32 :17-19, timestep_embedding :103-121).

Parameters live in a flat dict keyed exactly like the reference
``state_dict`` so that reference checkpoints load unchanged.
"""
import math

import torch
import torch.nn.functional as F


def topology(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2,
             channel_mult=(1, 2, 2, 4, 4), resblock_updown=True):
    """List of blocks in execution order.

    Each entry is a dict: kind in {"conv_in", "res", "down", "up", "out"},
    key prefix, cin/cout, updown in {None, "down", "up"}, and for decoder
    blocks ``concat`` = channels popped from the skip stack.  With
    resblock_updown=False the resampling layers are Downsample(use_conv=True)
    (kind "down": stride-2 Conv3d, prefix ...op) and Upsample(use_conv=True)
    (kind "up": nearest x2 + Conv3d, prefix ...conv), unet.py:40-100, :606-612, :700-706.
    """
    blocks = [dict(kind="conv_in", prefix="input_blocks.0.0", cin=in_channels, cout=model_channels)]
    chans = [model_channels]
    ch = model_channels
    idx = 1
    for level, mult in enumerate(channel_mult):
        for _ in range(num_res_blocks):
            blocks.append(dict(kind="res", prefix=f"input_blocks.{idx}.0", cin=ch, cout=mult * model_channels,
                               updown=None, push=True))
            ch = mult * model_channels
            chans.append(ch)
            idx += 1
        if level != len(channel_mult) - 1:
            if resblock_updown:
                blocks.append(dict(kind="res", prefix=f"input_blocks.{idx}.0", cin=ch, cout=ch, updown="down",
                                   push=True))
            else:
                blocks.append(dict(kind="down", prefix=f"input_blocks.{idx}.0.op", cin=ch, cout=ch, push=True))
            chans.append(ch)
            idx += 1
    blocks.append(dict(kind="res", prefix="middle_block.0", cin=ch, cout=ch, updown=None))
    blocks.append(dict(kind="res", prefix="middle_block.1", cin=ch, cout=ch, updown=None))
    idx = 0
    for level, mult in list(enumerate(channel_mult))[::-1]:
        for i in range(num_res_blocks + 1):
            ich = chans.pop()
            mid = model_channels * mult
            blocks.append(dict(kind="res", prefix=f"output_blocks.{idx}.0", cin=ch + ich, cout=mid,
                               updown=None, pop=ich))
            ch = mid
            if level and i == num_res_blocks:
                if resblock_updown:
                    blocks.append(dict(kind="res", prefix=f"output_blocks.{idx}.1", cin=ch, cout=ch, updown="up"))
                else:
                    blocks.append(dict(kind="up", prefix=f"output_blocks.{idx}.1.conv", cin=ch, cout=ch))
            idx += 1
    blocks.append(dict(kind="out", prefix="out", cin=ch, cout=out_channels))
    return blocks


def param_shapes(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2,
                 channel_mult=(1, 2, 2, 4, 4), resblock_updown=True):
    """Ordered (name, shape) list matching the reference state_dict."""
    ted = 4 * model_channels
    out = [("time_embed.0.weight", (ted, model_channels)), ("time_embed.0.bias", (ted,)),
           ("time_embed.2.weight", (ted, ted)), ("time_embed.2.bias", (ted,))]
    for b in topology(in_channels, model_channels, out_channels, num_res_blocks, channel_mult, resblock_updown):
        p, ci, co = b["prefix"], b["cin"], b["cout"]
        if b["kind"] in ("conv_in", "down", "up"):
            out += [(p + ".weight", (co, ci, 3, 3, 3)), (p + ".bias", (co,))]
        elif b["kind"] == "res":
            out += [(p + ".in_layers.0.weight", (ci,)), (p + ".in_layers.0.bias", (ci,)),
                    (p + ".in_layers.2.weight", (co, ci, 3, 3, 3)), (p + ".in_layers.2.bias", (co,)),
                    (p + ".emb_layers.1.weight", (co, ted)), (p + ".emb_layers.1.bias", (co,)),
                    (p + ".out_layers.0.weight", (co,)), (p + ".out_layers.0.bias", (co,)),
                    (p + ".out_layers.3.weight", (co, co, 3, 3, 3)), (p + ".out_layers.3.bias", (co,))]
            if ci != co:
                out += [(p + ".skip_connection.weight", (co, ci, 1, 1, 1)), (p + ".skip_connection.bias", (co,))]
        else:
            out += [(p + ".0.weight", (ci,)), (p + ".0.bias", (ci,)),
                    (p + ".2.weight", (co, ci, 3, 3, 3)), (p + ".2.bias", (co,))]
    return out


def random_params(seed=1, std=0.05, **cfg):
    """Seeded non-degenerate weights (the reference's zero-init
    layers would make every parity test vacuous).  GroupNorm gammas are drawn
    around 1, everything else N(0, std)."""
    g = torch.Generator().manual_seed(seed)
    params = {}
    for name, shape in param_shapes(**cfg):
        if len(shape) == 1 and (".in_layers.0." in name or ".out_layers.0." in name or name.startswith("out.0.")):
            base = 1.0 if name.endswith("weight") else 0.0
            params[name] = base + 0.1 * torch.randn(shape, generator=g)
        else:
            fan_in = 1
            for s in shape[1:]:
                fan_in *= s
            scale = std if len(shape) == 1 else min(std, 1.0 / math.sqrt(max(fan_in, 1)) * 1.5)
            params[name] = scale * torch.randn(shape, generator=g)
    return params


def timestep_embedding(t, dim, max_period=10000):
    """nn.py:103-121 (cos first, then sin)."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def _gn_silu(x, w, b, groups):
    return F.silu(F.group_norm(x.float(), groups, w, b, eps=1e-5).type(x.dtype))


def _resblock(P, p, x, emb, groups, updown):
    """ResBlock._forward (unet.py:285-311)."""
    h = _gn_silu(x, P[p + ".in_layers.0.weight"], P[p + ".in_layers.0.bias"], groups)
    if updown == "down":
        h = F.avg_pool3d(h, kernel_size=2, stride=2)
        x = F.avg_pool3d(x, kernel_size=2, stride=2)
    elif updown == "up":
        h = F.interpolate(h, scale_factor=2, mode="nearest")
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    h = F.conv3d(h, P[p + ".in_layers.2.weight"], P[p + ".in_layers.2.bias"], padding=1)
    e = F.linear(F.silu(emb), P[p + ".emb_layers.1.weight"], P[p + ".emb_layers.1.bias"])
    h = h + e[:, :, None, None, None]
    h = _gn_silu(h, P[p + ".out_layers.0.weight"], P[p + ".out_layers.0.bias"], groups)
    h = F.conv3d(h, P[p + ".out_layers.3.weight"], P[p + ".out_layers.3.bias"], padding=1)
    if (p + ".skip_connection.weight") in P:
        x = F.conv3d(x, P[p + ".skip_connection.weight"], P[p + ".skip_connection.bias"])
    return x + h


def unet_forward(P, x, t, model_channels=64, num_groups=32, in_channels=32, out_channels=8,
                 num_res_blocks=2, channel_mult=(1, 2, 2, 4, 4), trace=None, resblock_updown=True):
    """UNetModel.forward (unet.py:754-800).  ``trace`` (optional list)
    collects every block output for layer-level parity tests."""
    emb = timestep_embedding(t, model_channels)
    emb = F.linear(emb, P["time_embed.0.weight"], P["time_embed.0.bias"])
    emb = F.linear(F.silu(emb), P["time_embed.2.weight"], P["time_embed.2.bias"])
    hs = []
    h = x
    for b in topology(in_channels, model_channels, out_channels, num_res_blocks, channel_mult, resblock_updown):
        p = b["prefix"]
        if b["kind"] == "conv_in":
            h = F.conv3d(h, P[p + ".weight"], P[p + ".bias"], padding=1)
            hs.append(h)
        elif b["kind"] == "down":     # Downsample(use_conv=True): conv_nd(3, C, C, 3, stride=2, padding=1)
            h = F.conv3d(h, P[p + ".weight"], P[p + ".bias"], stride=2, padding=1)
            hs.append(h)
        elif b["kind"] == "up":       # Upsample(use_conv=True): nearest x2, then conv_nd(3, C, C, 3, padding=1)
            h = F.conv3d(F.interpolate(h, scale_factor=2, mode="nearest"), P[p + ".weight"], P[p + ".bias"],
                         padding=1)
        elif b["kind"] == "res":
            if "pop" in b:
                h = torch.cat([h, hs.pop()], dim=1)
            h = _resblock(P, p, h, emb, num_groups, b["updown"])
            if b.get("push"):
                hs.append(h)
        else:
            h = _gn_silu(h, P[p + ".0.weight"], P[p + ".0.bias"], num_groups)
            h = F.conv3d(h, P[p + ".2.weight"], P[p + ".2.bias"], padding=1)
        if trace is not None:
            trace.append(h)
    return h


class OracleUNet:
    """Callable ``model(x, t)`` seam around unet_forward."""

    def __init__(self, params, **cfg):
        self.P = params
        self.cfg = cfg

    def __call__(self, x, t, **kw):
        with torch.no_grad():
            return unet_forward(self.P, x, t, **self.cfg)
