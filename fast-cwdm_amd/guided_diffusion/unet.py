"""UNetModel on the native U-Net plan (drop-in for guided_diffusion/unet.py:451-800).

Constructor arguments, parameter names/shapes (state_dict) and the
``forward(x, timesteps, y=None)`` contract are the reference's; the forward
runs as one call into libcwdm (``cwdm_unet_forward``): time embedding, 35
ResBlocks and the output head become ~160 fused launches (GroupNorm-finalize +
implicit-GEMM Conv3d on MFMA with GN/SiLU/pool/upsample/concat/skip/bias/
residual folded in).  Activations are channels-last NDHWC in the
compute dtype (``compute_dtype`` = "fp32" for reference numerics, "bf16" for
throughput); parameters stay fp32 masters and are re-packed when they change.

Supported configuration family: the one run.sh uses (dims=3, no attention,
resblock_updown=True, use_scale_shift_norm=False, additive_skips=False,
resample_2d=False).  Anything else raises NotImplementedError at construction.
"""
import math
import os

import torch as th
import torch.nn as nn

from cwdm_hip import ops
from cwdm_hip.unet_runtime import UNetPlan


def _register(root, dotted, param):
    parts = dotted.split(".")
    mod = root
    for p in parts[:-1]:
        if p not in mod._modules:
            mod.add_module(p, nn.Module())
        mod = mod._modules[p]
    mod.register_parameter(parts[-1], param)


class UNetModel(nn.Module):
    def __init__(
        self,
        image_size,
        in_channels,
        model_channels,
        out_channels,
        num_res_blocks,
        attention_resolutions,
        dropout=0,
        channel_mult=(1, 2, 4, 8),
        conv_resample=True,
        dims=2,
        num_classes=None,
        use_checkpoint=False,
        use_fp16=False,
        num_heads=1,
        num_head_channels=-1,
        num_heads_upsample=-1,
        use_scale_shift_norm=False,
        resblock_updown=False,
        use_new_attention_order=False,
        num_groups=32,
        bottleneck_attention=True,
        resample_2d=True,
        additive_skips=False,
        decoder_device_thresh=0,
        compute_dtype=None,
    ):
        super().__init__()
        unsupported = []
        if dims != 3:
            unsupported.append(f"dims={dims} (3D only)")
        if attention_resolutions:
            unsupported.append("attention blocks")
        if bottleneck_attention:
            unsupported.append("bottleneck_attention=True")
        if not resblock_updown:
            unsupported.append("resblock_updown=False")
        if use_scale_shift_norm:
            unsupported.append("use_scale_shift_norm=True")
        if additive_skips:
            unsupported.append("additive_skips=True")
        if resample_2d:
            unsupported.append("resample_2d=True")
        if num_classes is not None:
            unsupported.append("class conditioning")
        if dropout:
            unsupported.append("dropout > 0")
        if unsupported:
            raise NotImplementedError("fast-cwdm_amd UNetModel covers the run.sh configuration only; unsupported: "
                                      + ", ".join(unsupported))
        self.image_size = image_size
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.attention_resolutions = attention_resolutions
        self.dropout = dropout
        self.channel_mult = tuple(channel_mult)
        self.conv_resample = conv_resample
        self.num_classes = num_classes
        self.use_checkpoint = use_checkpoint
        self.num_heads = num_heads
        self.num_groups = num_groups
        self.bottleneck_attention = bottleneck_attention
        self.additive_skips = additive_skips
        self.decoder_device_thresh = decoder_device_thresh
        self.devices = None
        if compute_dtype is None:
            compute_dtype = os.environ.get("CWDM_COMPUTE_DTYPE", "fp32")
        self.compute_dtype = compute_dtype
        self._plans = {}
        spec_plan = self._plan(compute_dtype)
        for name, shape in spec_plan.param_specs:
            _register(self, name, nn.Parameter(th.empty(shape, dtype=th.float32)))
        self._reset_parameters()
        self._packed = None
        self._packed_key = None

    # ---- parameters -------------------------------------------------------
    def _reset_parameters(self):
        """PyTorch default init of Conv3d/Linear/GroupNorm plus the reference's
        zero_module on out_layers.3 and out.2 (unet.py:259-261, :724)."""
        with th.no_grad():
            for name, p in self.named_parameters():
                if name.endswith("out_layers.3.weight") or name.endswith("out_layers.3.bias") or \
                        name.startswith("out.2."):
                    p.zero_()
                elif p.dim() == 1 and (".in_layers.0." in name or ".out_layers.0." in name or name.startswith("out.0.")):
                    p.fill_(1.0 if name.endswith("weight") else 0.0)
                elif p.dim() >= 2:
                    fan_in = p[0].numel()
                    bound = 1.0 / math.sqrt(fan_in)
                    p.uniform_(-bound, bound)
                else:
                    wname = name[: -len("bias")] + "weight"
                    w = dict(self.named_parameters())[wname]
                    bound = 1.0 / math.sqrt(w[0].numel())
                    p.uniform_(-bound, bound)

    def _plan(self, dtype):
        key = str(dtype)
        if key not in self._plans:
            self._plans[key] = UNetPlan(self.in_channels, self.model_channels, self.out_channels,
                                        self.num_res_blocks, self.channel_mult, self.num_groups, dtype)
        return self._plans[key]

    @property
    def plan(self):
        return self._plan(self.compute_dtype)

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self._packed = None
        return self

    def packed_weights(self):
        """Packed kernel-layout weights; re-packed whenever a parameter changed."""
        params = list(self.parameters())
        key = (self.compute_dtype,) + tuple((p.data_ptr(), p._version) for p in params)
        if self._packed is None or self._packed_key != key:
            ops._need_cuda(*params)
            flat = [p.detach().float().contiguous() for p in params]
            self._packed = self.plan.pack(flat)
            self._packed_key = key
        return self._packed

    def to(self, *args, **kwargs):
        """Reference semantics, except that a device list (the 2-GPU layer split
        of unet.py:727-752) places the whole model on the first device: on
        MI355X one GPU holds the model and the 128^3 activations many times over."""
        if args and isinstance(args[0], (list, tuple)):
            devs = list(args[0])
            super().to(devs[0])
            self.devices = [th.device(devs[0]), th.device(devs[0])]
            return self
        super().to(*args, **kwargs)
        p = next(self.parameters())
        self.devices = [p.device, p.device]
        return self

    # ---- forward ------------------------------------------------------------
    def forward_ndhwc(self, x_ndhwc, t_f32, out_ndhwc):
        """Fast seam: x (B, D, H, W, in) in the compute dtype, t fp32[B] (model
        timesteps), out (B, D, H, W, out) fp32; all device tensors."""
        B, D, H, W, C = x_ndhwc.shape
        assert C == self.in_channels
        return self.plan.forward(self.packed_weights(), x_ndhwc, t_f32, out_ndhwc, B, D, H, W)

    def forward(self, x, timesteps, y=None):
        assert (y is not None) == (self.num_classes is not None), \
            "must specify y if and only if the model is class-conditional"
        ops._need_cuda(x, timesteps)
        if self.devices is not None:
            assert x.device == self.devices[0], f"{x.device=} does not match {self.devices[0]=}"
        B, C, D, H, W = x.shape
        assert C == self.in_channels
        plan = self.plan
        plan.check_grid(D, H, W)
        V = D * H * W
        xin = th.empty((B, D, H, W, C), dtype=plan.torch_dtype, device=x.device)
        ops.copy3(x.contiguous().float() if x.dtype not in (th.float32, th.bfloat16) else x.contiguous(),
                  (C * V, V, 1), xin, (V * C, 1, C), B, C, V)
        t = timesteps.to(device=x.device, dtype=th.float32).contiguous()
        out_nd = th.empty((B, D, H, W, self.out_channels), dtype=th.float32, device=x.device)
        self.forward_ndhwc(xin, t, out_nd)
        out = th.empty((B, self.out_channels, D, H, W), dtype=th.float32, device=x.device)
        oc = self.out_channels
        ops.copy3(out_nd, (V * oc, 1, oc), out, (oc * V, V, 1), B, oc, V)
        return out
