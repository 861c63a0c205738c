"""Oracle: functional WavUNetModel (use_freq=True) (TEST INFRASTRUCTURE ONLY).

Restates guided_diffusion/wunet.py of the reference for the configuration
script_util.create_model builds with use_freq=True (:268-292): no attention,
bottleneck_attention off, resblock_updown=True, progressive_input='residual',
use_scale_shift_norm=False, dropout 0:
* ResBlock (:148-269): in_layers (GN, SiLU, Conv3d) at the INPUT resolution;
  down=True: Downsample(use_freq) = DWT of the conv output and of x, LLL / 3,
  the conv output's 7 high bands are returned as the skip (:120-128, :239-245);
  up=True: Upsample(use_freq) = IDWT(3 h, skip bands) (:40-80); then + emb,
  out_layers at the output resolution, skip_connection + h.
* WaveletDownsample (:131-145): conv(cat(8 DWT bands) / 3) of the input
  pyramid, added to h after every downsampling ResBlock.
* The decoder is built with the reference's list reuse (:648-687): the block
  closing a level is Sequential(<the level's last ResBlock again>, up ResBlock),
  so that ResBlock's weights appear under two state_dict prefixes and it runs
  twice.  Reproduced, as is the skip routing of forward (:754-795).
Haar by oracle.haar (pinned to PyWavelets); every tensor fp32 NCDHW.
"""
import torch
import torch.nn.functional as F

from . import haar
from .unet import _gn_silu, timestep_embedding


def topology(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2, channel_mult=(1, 2, 2, 4, 4)):
    """Execution list.  Entries: ("conv_in", prefix, cin, cout), ("res", prefix, cin, cout, updown),
    ("pyr", prefix, cin, cout) (WaveletDownsample), ("dec", [entries...]) (one output block),
    ("out", prefix, cin, cout)."""
    mc, nrb = model_channels, num_res_blocks
    ent = [("conv_in", "input_blocks.0.0", in_channels, mc)]
    ch, pyr, idx = mc, in_channels, 1
    for mult in channel_mult:
        for _ in range(nrb):
            ent.append(("res", f"input_blocks.{idx}.0", ch, mult * mc, None))
            ch = mult * mc
            idx += 1
        ent.append(("res", f"input_blocks.{idx}.0", ch, ch, "down"))
        ent.append(("pyr", f"input_blocks.{idx + 1}.0", pyr, ch))
        pyr = ch
        idx += 2
    ent.append(("res", "middle_block.0", ch, ch, None))
    ent.append(("res", "middle_block.1", ch, ch, None))
    idx = 0
    for mult in reversed(channel_mult):
        layers = []
        for i in range(nrb + 1):
            if i != nrb:
                mid = mc * mult
                layers = [("res", f"output_blocks.{idx}.0", ch, mid, None)]
                ch = mid
            else:
                prev = layers[0]
                layers = [("res", f"output_blocks.{idx}.0", prev[2], prev[3], None, prev[1]),   # alias of prev
                          ("res", f"output_blocks.{idx}.1", ch, ch, "up")]
            ent.append(("dec", layers))
            idx += 1
    for i in range(nrb):
        ent.append(("res", f"out_res.{i}.0", ch, ch, None))
    ent.append(("out", "out", ch, out_channels))
    return ent


def _res_params(p, ci, co, ted):
    out = [(p + ".in_layers.0.weight", (ci,)), (p + ".in_layers.0.bias", (ci,)),
           (p + ".in_layers.2.weight", (co, ci, 3, 3, 3)), (p + ".in_layers.2.bias", (co,)),
           (p + ".emb_layers.1.weight", (co, ted)), (p + ".emb_layers.1.bias", (co,)),
           (p + ".out_layers.0.weight", (co,)), (p + ".out_layers.0.bias", (co,)),
           (p + ".out_layers.3.weight", (co, co, 3, 3, 3)), (p + ".out_layers.3.bias", (co,))]
    if ci != co:
        out += [(p + ".skip_connection.weight", (co, ci, 1, 1, 1)), (p + ".skip_connection.bias", (co,))]
    return out


def param_shapes(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2, channel_mult=(1, 2, 2, 4, 4),
                 with_aliases=False):
    """Ordered (name, shape) of the reference state_dict.  with_aliases adds the
    second prefix of each reused decoder ResBlock (state_dict lists both)."""
    ted = 4 * model_channels
    out = [("time_embed.0.weight", (ted, model_channels)), ("time_embed.0.bias", (ted,)),
           ("time_embed.2.weight", (ted, ted)), ("time_embed.2.bias", (ted,))]
    for e in topology(in_channels, model_channels, out_channels, num_res_blocks, channel_mult):
        if e[0] == "conv_in":
            out += [(e[1] + ".weight", (e[3], e[2], 3, 3, 3)), (e[1] + ".bias", (e[3],))]
        elif e[0] == "res":
            out += _res_params(e[1], e[2], e[3], ted)
        elif e[0] == "pyr":
            out += [(e[1] + ".conv.weight", (e[3], 8 * e[2], 3, 3, 3)), (e[1] + ".conv.bias", (e[3],))]
        elif e[0] == "dec":
            for r in e[1]:
                if len(r) == 6:
                    if with_aliases:
                        out += _res_params(r[1], r[2], r[3], ted)
                else:
                    out += _res_params(r[1], r[2], r[3], ted)
        else:
            out += [(e[1] + ".0.weight", (e[2],)), (e[1] + ".0.bias", (e[2],)),
                    (e[1] + ".2.weight", (e[3], e[2], 3, 3, 3)), (e[1] + ".2.bias", (e[3],))]
    return out


def aliases(**cfg):
    """{alias prefix: owner prefix} of the reused decoder ResBlocks."""
    out = {}
    for e in topology(**cfg):
        if e[0] == "dec":
            for r in e[1]:
                if len(r) == 6:
                    out[r[1]] = r[5]
    return out


def random_params(seed=1, std=0.05, **cfg):
    import math
    g = torch.Generator().manual_seed(seed)
    params = {}
    for name, shape in param_shapes(**cfg):
        if len(shape) == 1 and (".in_layers.0." in name or ".out_layers.0." in name or name.startswith("out.0.")):
            params[name] = (1.0 if name.endswith("weight") else 0.0) + 0.1 * torch.randn(shape, generator=g)
        else:
            fan_in = 1
            for s in shape[1:]:
                fan_in *= s
            scale = std if len(shape) == 1 else min(std, 1.0 / math.sqrt(max(fan_in, 1)) * 1.5)
            params[name] = scale * torch.randn(shape, generator=g)
    return params


def _cat_bands(bands):
    return torch.cat(list(bands), dim=1)


def _resblock(P, p, x, skip, emb, groups, updown):
    """wunet.ResBlock.forward (:210-269); returns (out, hSkip)."""
    h = _gn_silu(x, P[p + ".in_layers.0.weight"], P[p + ".in_layers.0.bias"], groups)
    h = F.conv3d(h, P[p + ".in_layers.2.weight"], P[p + ".in_layers.2.bias"], padding=1)
    if updown == "down":
        hb = haar.dwt3d(h)
        xb = haar.dwt3d(x)
        h, skip = hb[0] / 3.0, tuple(hb[1:])
        x = xb[0] / 3.0
    elif updown == "up":
        h = haar.idwt3d(3.0 * h, *skip)
        x = haar.idwt3d(3.0 * x, *skip)
    e = F.linear(F.silu(emb), P[p + ".emb_layers.1.weight"], P[p + ".emb_layers.1.bias"])
    h = h + e[:, :, None, None, None]
    h = _gn_silu(h, P[p + ".out_layers.0.weight"], P[p + ".out_layers.0.bias"], groups)
    h = F.conv3d(h, P[p + ".out_layers.3.weight"], P[p + ".out_layers.3.bias"], padding=1)
    if (p + ".skip_connection.weight") in P:
        x = F.conv3d(x, P[p + ".skip_connection.weight"], P[p + ".skip_connection.bias"])
    return x + h, skip


def wunet_forward(P, x, t, model_channels=64, num_groups=32, in_channels=32, out_channels=8, num_res_blocks=2,
                  channel_mult=(1, 2, 2, 4, 4), trace=None):
    """WavUNetModel.forward (wunet.py:754-795)."""
    cfg = dict(in_channels=in_channels, model_channels=model_channels, out_channels=out_channels,
               num_res_blocks=num_res_blocks, channel_mult=channel_mult)
    emb = timestep_embedding(t, model_channels)
    emb = F.linear(emb, P["time_embed.0.weight"], P["time_embed.0.bias"])
    emb = F.linear(F.silu(emb), P["time_embed.2.weight"], P["time_embed.2.bias"])
    hs = []
    pyr = x
    h = x
    skip = None
    for e in topology(**cfg):
        kind = e[0]
        if kind == "conv_in":
            h = F.conv3d(h, P[e[1] + ".weight"], P[e[1] + ".bias"], padding=1)
            hs.append(None)
        elif kind == "res" and e[1].startswith("input_blocks"):
            h, sk = _resblock(P, e[1], h, None, emb, num_groups, e[4])
            hs.append(sk if e[4] == "down" else None)
        elif kind == "pyr":
            pb = _cat_bands(haar.dwt3d(pyr)) / 3.0
            pyr = F.conv3d(pb, P[e[1] + ".conv.weight"], P[e[1] + ".conv.bias"], padding=1) + h
            h = pyr
        elif kind == "res" and e[1].startswith("middle_block"):
            h, _ = _resblock(P, e[1], h, None, emb, num_groups, None)
        elif kind == "dec":
            new = hs.pop()
            if new is not None:
                skip = new
            for r in e[1]:
                owner = r[5] if len(r) == 6 else r[1]
                h, _ = _resblock(P, owner, h, skip, emb, num_groups, r[4])
        elif kind == "res":       # out_res
            h, _ = _resblock(P, e[1], h, skip, emb, num_groups, None)
        else:
            h = _gn_silu(h, P[e[1] + ".0.weight"], P[e[1] + ".0.bias"], num_groups)
            h = F.conv3d(h, P[e[1] + ".2.weight"], P[e[1] + ".2.bias"], padding=1)
        if trace is not None and kind != "dec":
            trace.append(h)
        elif trace is not None:
            trace.append(h)
    return h
