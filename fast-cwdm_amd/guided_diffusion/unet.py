"""UNetModel on the native U-Net plan (drop-in for guided_diffusion/unet.py:451-800).

Constructor arguments, parameter names/shapes (state_dict) and the
``forward(x, timesteps, y=None)`` contract are the reference's; the forward
runs as one call into libcwdm (``cwdm_unet_forward``): time embedding, 35
ResBlocks and the output head become ~160 fused launches (GroupNorm-finalize +
implicit-GEMM Conv3d on MFMA with GN/SiLU/pool/upsample/concat/skip/bias/
residual folded in).  Activations are channels-last NDHWC in the
compute dtype (``compute_dtype`` = "fp32" for reference numerics, "bf16" or
"fp16" for throughput -- the same MFMA rate on gfx950, fp16 with 3 more mantissa
bits); parameters stay fp32 masters and are re-packed when they change.

Supported configuration family: the one run.sh uses (dims=3, no attention,
use_scale_shift_norm=False, additive_skips=False, resample_2d=False), with
either resblock_updown=True (run.sh: ResBlock down/up) or resblock_updown=False
with conv_resample=True (Downsample = stride-2 Conv3d, Upsample = nearest x2 +
Conv3d; unet.py:40-100).  Anything else raises NotImplementedError.
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


_NO_PARAM_CACHE = os.environ.get("CWDM_PARAM_CACHE", "1") == "0"
# direct_grads training forward through one anchor input (env CWDM_GRAD_ANCHOR=0: the parameters, A/B knob)
_ANCHOR_ON = os.environ.get("CWDM_GRAD_ANCHOR", "1") != "0"

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
        if not resblock_updown and not conv_resample:
            unsupported.append("resblock_updown=False with conv_resample=False (parameter-free pool / nearest layers)")
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
        self._setup_native(image_size, in_channels, model_channels, out_channels, num_res_blocks,
                           attention_resolutions, dropout, channel_mult, conv_resample, num_classes, use_checkpoint,
                           num_heads, num_groups, resblock_updown, bottleneck_attention, additive_skips,
                           decoder_device_thresh, compute_dtype)

    use_freq = False

    def _setup_native(self, image_size, in_channels, model_channels, out_channels, num_res_blocks,
                      attention_resolutions, dropout, channel_mult, conv_resample, num_classes, use_checkpoint,
                      num_heads, num_groups, resblock_updown, bottleneck_attention, additive_skips,
                      decoder_device_thresh, compute_dtype):
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
        self.resblock_updown = bool(resblock_updown)
        self.bottleneck_attention = bottleneck_attention
        self.additive_skips = additive_skips
        self.decoder_device_thresh = decoder_device_thresh
        self.devices = None
        if compute_dtype is None:
            compute_dtype = os.environ.get("CWDM_COMPUTE_DTYPE", "fp32")
        self.compute_dtype = compute_dtype
        self._plans = {}
        spec_plan = self._plan(compute_dtype)
        # state_dict order; a reused block's second names (WavUNetModel) alias the owner's Parameter
        by_pos = {}
        for name, owner, before in spec_plan.aliases:
            by_pos.setdefault(before, []).append((name, owner))
        registered = []
        specs = spec_plan.param_specs
        for i in range(len(specs) + 1):
            for aname, owner in by_pos.get(i, []):
                _register(self, aname, registered[owner])
            if i < len(specs):
                registered.append(nn.Parameter(th.empty(specs[i][1], dtype=th.float32)))
                _register(self, specs[i][0], registered[-1])
        self._reset_parameters()
        self._param_gen = 0
        self._packed = None
        self._packed_key = None
        self._packed_bwd = None
        self._packed_bwd_key = None
        self._src_ptrs = None      # (data_ptrs, ctypes pointer array) of the fp32 parameter views
        self._grad_hook = None       # called per backward segment (DDP bucket all-reduce)
        self._last_grad_flat = None
        # training forward keeps the DMA-staged convs' activated inputs (more
        # workspace, no GroupNorm+SiLU recompute in the weight gradients)
        self.keep_activations = True
        # backward assigns .grad = views of the flat gradient buffer directly
        # (TrainLoop turns it on); off, the views are returned to autograd, so
        # torch.autograd.grad and backward(inputs=...) behave as usual
        self.direct_grads = False
        self._flatten_params()

    # ---- flat parameter storage ---------------------------------------------
    def _flatten_params(self):
        """All parameters become views of ONE contiguous fp32 buffer (state_dict
        order): the optimizer, gradient all-reduce and weight packing run over
        flat ranges; the views share the buffer's version counter."""
        params = list(self.parameters())
        # the hot paths (forward, packs, backward, zero_grad) read this list: a
        # traversal of the module tree per call cost ~0.2-0.3 ms of host time,
        # several per training step, while the GPU waited at the step's start
        # (parameters are views of the flat buffer, never re-registered after
        # construction; _apply re-flattens and refreshes it)
        self._param_list = params
        if not params:
            return
        dev = params[0].device
        flat = th.empty(sum(p.numel() for p in params), dtype=th.float32, device=dev)
        o = 0
        with th.no_grad():
            for p in params:
                n = p.numel()
                flat[o:o + n].copy_(p.data.reshape(-1))
                p.data = flat[o:o + n].view(p.shape)
                o += n
        self._flat = flat

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self._flatten_params()
        self._packed = self._packed_bwd = None
        return r

    @property
    def flat_params(self):
        return self._flat

    def param_list(self):
        """The parameters in registration (state_dict) order, cached (env
        CWDM_PARAM_CACHE=0: a fresh traversal per call, A/B knob)."""
        if _NO_PARAM_CACHE:
            return list(self.parameters())
        pl = self.__dict__.get("_param_list")
        if pl is None:
            pl = self._param_list = list(self.parameters())
        return pl

    def flat_grad(self):
        """Flat fp32 gradient of the last backward (the buffer the native backward
        wrote when the .grad tensors still alias it, else a concatenation)."""
        params = self.param_list()
        g = self._last_grad_flat
        if g is not None and params[0].grad is not None and params[0].grad.data_ptr() == g.data_ptr() and \
                params[-1].grad.data_ptr() == g[g.numel() - params[-1].numel():].data_ptr():
            return g
        return th.cat([(p.grad if p.grad is not None else th.zeros_like(p)).reshape(-1) for p in params])

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
                                        self.num_res_blocks, self.channel_mult, self.num_groups, dtype,
                                        resblock_updown=self.resblock_updown, use_freq=self.use_freq)
        return self._plans[key]

    @property
    def plan(self):
        return self._plan(self.compute_dtype)

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        # both packed layouts are per dtype (the plan's packed sizes differ)
        self._packed = self._packed_bwd = None
        self._packed_key = self._packed_bwd_key = None
        return self

    def mark_params_changed(self):
        """Tell the model its parameters were written behind autograd's back
        (raw-pointer kernels, collectives into ``p.data``): the next forward /
        backward re-packs the kernel-layout weights."""
        self._param_gen += 1

    def _weights_key(self):
        # parameters are views of self._flat but each has its own version
        # counter (set_data); writers of the flat buffer bump the flat's, in-place
        # ops on a parameter bump that parameter's, raw writers call
        # mark_params_changed -- the key covers all three
        params = self.param_list()
        return (self.compute_dtype, self._param_gen, self._flat._version) + \
            tuple((p.data_ptr(), p._version) for p in params)

    def packed_weights(self):
        """Packed kernel-layout weights; re-packed whenever a parameter changed."""
        params = self.param_list()
        key = self._weights_key()
        if self._packed is None or self._packed_key != key:
            arr = self._src_array(params, key)
            flat = params if arr is not None else [p.detach().float().contiguous() for p in params]
            # re-pack in place (stream-ordered after earlier readers; a captured
            # sampling graph keeps a valid pointer; the plan's batched pack job
            # table stays cached when no pointer moved)
            old = self._packed if (self._packed is not None and self._packed.device == flat[0].device) else None
            self._packed = self.plan.pack(flat, packed=old, arr=arr)
            self._packed_key = key
        return self._packed

    def _src_array(self, params, key):
        """The parameters' pointer array for the packs, cached while no pointer
        moved: every training step re-packs, and building the per-parameter
        views and the array each time cost ~1 ms of host time per step, during
        which the GPU idled.  None when a parameter is not an fp32 contiguous
        CUDA tensor (the pack then reads converted copies)."""
        ptrs = tuple(k[0] for k in key[3:])
        if self._src_ptrs is not None and self._src_ptrs[0] == ptrs:
            return self._src_ptrs[1]
        ops._need_cuda(*params)
        if not all(p.dtype == th.float32 and p.is_contiguous() for p in params):
            return None
        arr = self.plan.pointer_array(params)
        self._src_ptrs = (ptrs, arr)
        return arr

    def packed_bwd_weights(self):
        """Transposed/flipped dgrad weight layouts for the native backward."""
        params = self.param_list()
        key = self._weights_key()
        if self._packed_bwd is None or self._packed_bwd_key != key:
            arr = self._src_array(params, key)
            old = self._packed_bwd if (self._packed_bwd is not None and
                                       self._packed_bwd.device == params[0].device) else None
            src = params if arr is not None else [p.detach() for p in params]
            self._packed_bwd = self.plan.pack_bwd(src, packed_bwd=old, arr=arr)
            self._packed_bwd_key = key
        return self._packed_bwd

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

    def forward_step_ndhwc(self, x_ndhwc, t_f32, step):
        """forward_ndhwc followed by the sampling step ``step`` (ops.sampler_args,
        model_out = the (B, D, H, W, out) fp32 buffer), fused into the output
        head when it qualifies; returns whether it was fused."""
        B, D, H, W, C = x_ndhwc.shape
        assert C == self.in_channels
        return self.plan.forward_step(self.packed_weights(), x_ndhwc, t_f32, step, B, D, H, W)

    def forward(self, x, timesteps, y=None):
        assert (y is not None) == (self.num_classes is not None), \
            "must specify y if and only if the model is class-conditional"
        ops._need_cuda(x, timesteps)
        if self.devices is not None:
            assert x.device == self.devices[0], f"{x.device=} does not match {self.devices[0]=}"
        B, C, D, H, W = x.shape
        assert C == self.in_channels
        params = self.param_list()
        if th.is_grad_enabled() and any(p.requires_grad for p in params):
            if self.direct_grads and _ANCHOR_ON and all(p.grad is None for p in params):
                # every .grad is assigned by the backward itself (direct_grads, none to
                # accumulate into): one anchor input instead of the 230 parameters
                # (Function.apply's per-input autograd bookkeeping: ~0.23 ms of host
                # time per step, while the GPU waited at the step's start)
                anchor = self.__dict__.get("_grad_anchor")
                if anchor is None:
                    anchor = self._grad_anchor = th.zeros((), requires_grad=True)
                return _UNetTrain.apply(self, x, timesteps, anchor)
            return _UNetTrain.apply(self, x, timesteps, *params)
        xin, t = self._prep_inputs(x, timesteps)
        out_nd = th.empty((B, D, H, W, self.out_channels), dtype=th.float32, device=x.device)
        self.forward_ndhwc(xin, t, out_nd)
        return self._to_ncdhw(out_nd)

    def _prep_inputs(self, x, timesteps):
        B, C, D, H, W = x.shape
        plan = self.plan
        plan.check_grid(D, H, W)
        V = D * H * W
        xin = th.empty((B, D, H, W, C), dtype=plan.torch_dtype, device=x.device)
        ops.copy3(x.detach().contiguous().float() if x.dtype not in (th.float32, th.bfloat16, th.float16) else
                  x.detach().contiguous(), (C * V, V, 1), xin, (V * C, 1, C), B, C, V)
        t = timesteps.to(device=x.device, dtype=th.float32).contiguous()
        return xin, t

    def _to_ncdhw(self, out_nd):
        B, D, H, W, oc = out_nd.shape
        V = D * H * W
        out = th.empty((B, oc, D, H, W), dtype=th.float32, device=out_nd.device)
        ops.copy3(out_nd, (V * oc, 1, oc), out, (oc * V, V, 1), B, oc, V)
        return out


class _UNetTrain(th.autograd.Function):
    """Differentiable UNetModel.forward: the native forward keeps every
    activation in a private workspace; backward runs the native plan backward
    (cwdm_unet_backward) segment by segment, calling the model's grad hook
    after each so a data-parallel reducer can all-reduce finished gradient
    ranges while later segments compute."""

    @staticmethod
    def forward(ctx, model, x, timesteps, *params):
        ctx.anchored = len(params) == 1 and params[0] is model.__dict__.get("_grad_anchor")
        B, C, D, H, W = x.shape
        plan = model.plan
        xin, t = model._prep_inputs(x, timesteps)
        # the training workspace: the forward keeps each DMA-staged conv's
        # activated input there for the backward's weight gradients
        nbytes = plan.train_workspace_bytes(B, D, H, W) if model.keep_activations else \
            plan.workspace_bytes(B, D, H, W)
        ws = th.empty(nbytes, dtype=th.uint8, device=x.device)
        out_nd = th.empty((B, D, H, W, model.out_channels), dtype=th.float32, device=x.device)
        plan.forward(model.packed_weights(), xin, t, out_nd, B, D, H, W, ws=ws)
        ctx.model = model
        ctx.state = (xin, t, ws, (B, D, H, W))
        return model._to_ncdhw(out_nd)

    @staticmethod
    def backward(ctx, gout):
        model = ctx.model
        xin, t, ws, (B, D, H, W) = ctx.state
        ctx.state = None
        plan = model.plan
        oc = model.out_channels
        V = D * H * W
        dout = th.empty((B, D, H, W, oc), dtype=th.float32, device=xin.device)
        ops.copy3(gout.contiguous().float(), (oc * V, V, 1), dout, (V * oc, 1, oc), B, oc, V)
        grads = th.empty(plan.grad_numel, dtype=th.float32, device=xin.device)
        gws = th.empty(plan.grad_workspace_bytes(B, D, H, W), dtype=th.uint8, device=xin.device)
        packed, packed_bwd = model.packed_weights(), model.packed_bwd_weights()
        hook = model._grad_hook
        nseg = plan.num_segments
        if hook is None:
            plan.backward(packed, packed_bwd, xin, t, dout, grads, B, D, H, W, ws, gws, 0, nseg)
        else:
            for seg in range(nseg):
                plan.backward(packed, packed_bwd, xin, t, dout, grads, B, D, H, W, ws, gws, seg, seg + 1)
                off, n = plan.segment_range(seg)
                hook(seg, grads, off, n)
            hook(None, grads, 0, grads.numel())
        del ws, gws
        model._last_grad_flat = grads
        # with direct_grads, a parameter without a gradient gets its view of the
        # flat buffer as .grad directly (autograd would clone each returned view:
        # ~230 copies per step); otherwise (or with a gradient already there:
        # accumulation) the view is returned and autograd handles it as usual
        out = []
        o = 0
        for p, (_, shape) in zip(model.param_list(), plan.param_specs):
            n = 1
            for s_ in shape:
                n *= s_
            view = grads[o:o + n].view(shape)
            o += n
            if model.direct_grads and p.grad is None and p.requires_grad:
                p.grad = view
                out.append(None)
            elif ctx.anchored and p.requires_grad:
                p.grad.add_(view)   # (a .grad set between forward and backward: accumulate as autograd would)
                out.append(None)
            else:
                out.append(view)
        if ctx.anchored:
            return (None, None, None, None)
        return (None, None, None, *out)
