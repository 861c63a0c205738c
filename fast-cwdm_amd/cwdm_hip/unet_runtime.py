"""Python handle on the native U-Net plan (cwdm_unet_* in include/cwdm.h).

The plan (C++) owns the topology, the parameter naming contract and the launch
sequence; this wrapper only holds device buffers (packed weights, workspace)
allocated through torch's caching allocator.
"""
import ctypes

import torch

from . import _lib
from ._lib import CWDM_BF16, CWDM_F16, CWDM_F32, check, lib
from .ops import _need_cuda, _stream

_DTYPES = {"fp32": CWDM_F32, "float32": CWDM_F32, "bf16": CWDM_BF16, "bfloat16": CWDM_BF16,
           "fp16": CWDM_F16, "float16": CWDM_F16,
           # the accurate fast mode: fp32 storage, wide-grid conv MFMAs on bf16 hi/lo splits
           "fp32x": CWDM_F32}
SPLIT_DTYPES = ("fp32x",)
TORCH_DT = {CWDM_F32: torch.float32, CWDM_BF16: torch.bfloat16, CWDM_F16: torch.float16}


def parse_dtype(d):
    if isinstance(d, torch.dtype):
        d = {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float16: "fp16"}.get(d, str(d))
    if d not in _DTYPES:
        raise ValueError(f"compute dtype must be fp32, fp32x, bf16 or fp16, got {d!r}")
    return _DTYPES[d]


class UNetPlan:
    def __init__(self, in_channels, model_channels, out_channels, num_res_blocks, channel_mult, num_groups,
                 dtype="fp32", resblock_updown=True, use_freq=False):
        cfg = _lib.UNetConfig()
        cfg.in_channels, cfg.model_channels, cfg.out_channels = in_channels, model_channels, out_channels
        cfg.num_res_blocks, cfg.num_levels = num_res_blocks, len(channel_mult)
        if len(channel_mult) > 8:
            raise ValueError("at most 8 U-Net levels")
        for i, m in enumerate(channel_mult):
            cfg.channel_mult[i] = int(m)
        cfg.num_groups = num_groups
        cfg.dtype = parse_dtype(dtype)
        cfg.mfma_split = 1 if (isinstance(dtype, str) and dtype in SPLIT_DTYPES) else 0
        cfg.resblock_updown = 1 if resblock_updown else 0
        cfg.use_freq = 1 if use_freq else 0
        self.use_freq = bool(use_freq)
        self.dtype = cfg.dtype
        self.torch_dtype = TORCH_DT[cfg.dtype]
        self.num_levels = len(channel_mult)
        self.in_channels, self.out_channels = in_channels, out_channels
        h = ctypes.c_void_p()
        check(lib().cwdm_unet_create(ctypes.byref(cfg), ctypes.byref(h)), "UNetModel")
        self._h = h
        self._lib = lib()
        self.param_specs = []
        name = ctypes.create_string_buffer(256)
        shape = (ctypes.c_int64 * 5)()
        nd = ctypes.c_int()
        for i in range(lib().cwdm_unet_num_params(h)):
            check(lib().cwdm_unet_param_info(h, i, name, 256, shape, ctypes.byref(nd)))
            self.param_specs.append((name.value.decode(), tuple(shape[k] for k in range(nd.value))))
        # (alias name, owner index, index of the parameter it precedes in state_dict order)
        self.aliases = []
        owner, before = ctypes.c_int(), ctypes.c_int()
        for i in range(lib().cwdm_unet_num_aliases(h)):
            check(lib().cwdm_unet_alias_info(h, i, name, 256, ctypes.byref(owner), ctypes.byref(before)))
            self.aliases.append((name.value.decode(), owner.value, before.value))
        self._ws = None
        self._ws_key = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.cwdm_unet_destroy(h)
            self._h = None

    @property
    def packed_bytes(self):
        return int(lib().cwdm_unet_packed_bytes(self._h))

    def pointer_array(self, params):
        """ctypes array of the parameters' device pointers (param_specs order)."""
        if len(params) != len(self.param_specs):
            raise ValueError("parameter count mismatch")
        return (ctypes.c_void_p * len(params))(*[p.data_ptr() for p in params])

    def pack(self, params, packed=None, arr=None):
        """params: fp32 contiguous device tensors in param_specs order (arr: their
        pointer_array, already checked, when the caller keeps one)."""
        if len(params) != len(self.param_specs):
            raise ValueError("parameter count mismatch")
        dev = params[0].device
        # a buffer passed in is reused only when it holds this plan's layout
        # (the packed size depends on the compute dtype)
        if packed is None or packed.numel() < self.packed_bytes:
            packed = torch.empty(self.packed_bytes, dtype=torch.uint8, device=dev)
        if arr is None:
            _need_cuda(*params)
            arr = self.pointer_array(params)
        check(lib().cwdm_unet_pack(self._h, arr, ctypes.c_void_p(packed.data_ptr()), _stream()), "pack")
        return packed

    def workspace_bytes(self, B, D, H, W):
        n = int(lib().cwdm_unet_workspace_bytes(self._h, B, D, H, W))
        if n < 0:
            raise AssertionError("bad grid")
        return n

    def train_workspace_bytes(self, B, D, H, W):
        """Forward workspace that also keeps the convs' activated inputs for
        the DMA-staged weight gradients (cwdm_unet_train_workspace_bytes)."""
        n = int(lib().cwdm_unet_train_workspace_bytes(self._h, B, D, H, W))
        if n < 0:
            raise AssertionError("bad grid")
        return n

    def workspace(self, B, D, H, W, device):
        key = (B, D, H, W, str(device))
        if self._ws_key != key:
            self._ws = None
            self._ws = torch.empty(self.workspace_bytes(B, D, H, W), dtype=torch.uint8, device=device)
            self._ws_key = key
        return self._ws

    def check_grid(self, D, H, W):
        div = 2 ** (self.num_levels - (0 if self.use_freq else 1))
        if D % div or H % div or W % div:
            raise AssertionError(f"every subband edge must be divisible by {div} (got {D}x{H}x{W})")

    def forward(self, packed, x_ndhwc, t_f32, out_ndhwc, B, D, H, W, ws=None):
        _need_cuda(packed, x_ndhwc, t_f32, out_ndhwc)
        self.check_grid(D, H, W)
        if ws is None:
            ws = self.workspace(B, D, H, W, x_ndhwc.device)
        check(lib().cwdm_unet_forward(self._h, ctypes.c_void_p(packed.data_ptr()), ctypes.c_void_p(x_ndhwc.data_ptr()),
                                      ctypes.c_void_p(t_f32.data_ptr()), ctypes.c_void_p(out_ndhwc.data_ptr()),
                                      B, D, H, W, ctypes.c_void_p(ws.data_ptr()), ws.numel(), _stream()),
              "UNetModel.forward")
        return out_ndhwc

    def forward_step(self, packed, x_ndhwc, t_f32, step, B, D, H, W, ws=None):
        """cwdm_unet_forward_step: the forward plus the sampling step ``step``
        (an ops.sampler_args whose model_out is the NDHWC fp32 output buffer);
        returns True when the step ran fused into the output head."""
        _need_cuda(packed, x_ndhwc, t_f32)
        self.check_grid(D, H, W)
        if ws is None:
            ws = self.workspace(B, D, H, W, x_ndhwc.device)
        fused = ctypes.c_int(0)
        check(lib().cwdm_unet_forward_step(self._h, ctypes.c_void_p(packed.data_ptr()),
                                           ctypes.c_void_p(x_ndhwc.data_ptr()), ctypes.c_void_p(t_f32.data_ptr()),
                                           ctypes.byref(step), B, D, H, W, ctypes.c_void_p(ws.data_ptr()),
                                           ws.numel(), ctypes.byref(fused), _stream()),
              "UNetModel.forward_step")
        return bool(fused.value)

    def flops(self, B, D, H, W):
        return float(lib().cwdm_unet_flops(self._h, B, D, H, W))

    # ---- training -----------------------------------------------------------
    @property
    def grad_numel(self):
        n = 0
        for _, shape in self.param_specs:
            k = 1
            for s in shape:
                k *= s
            n += k
        return n

    @property
    def packed_bwd_bytes(self):
        return max(int(lib().cwdm_unet_packed_bwd_bytes(self._h)), 1)

    def pack_bwd(self, params, packed_bwd=None, arr=None):
        """Transposed/flipped (dgrad) weight layouts; re-run after every update."""
        need = self.packed_bwd_bytes
        if packed_bwd is None or packed_bwd.numel() < need:
            packed_bwd = torch.empty(need, dtype=torch.uint8, device=params[0].device)
        if arr is None:
            _need_cuda(*params)
            arr = self.pointer_array(params)
        check(lib().cwdm_unet_pack_bwd(self._h, arr, ctypes.c_void_p(packed_bwd.data_ptr()), _stream()), "pack_bwd")
        return packed_bwd

    def grad_workspace_bytes(self, B, D, H, W):
        n = int(lib().cwdm_unet_grad_workspace_bytes(self._h, B, D, H, W))
        if n < 0:
            raise AssertionError("bad grid")
        return n

    @property
    def num_segments(self):
        return int(lib().cwdm_unet_backward_segments(self._h))

    def segment_range(self, seg):
        off, n = ctypes.c_int64(), ctypes.c_int64()
        check(lib().cwdm_unet_segment_range(self._h, seg, ctypes.byref(off), ctypes.byref(n)))
        return off.value, n.value

    def backward(self, packed, packed_bwd, x_ndhwc, t_f32, dout_ndhwc, grads, B, D, H, W, ws, gws,
                 seg_begin=0, seg_end=None):
        """Gradients of all parameters (flat fp32 ``grads``) for the forward
        that last ran on ``ws``; ``dout_ndhwc`` fp32 (B, D, H, W, out)."""
        _need_cuda(packed, packed_bwd, x_ndhwc, t_f32, dout_ndhwc, grads, ws, gws)
        if seg_end is None:
            seg_end = self.num_segments
        assert grads.dtype == torch.float32 and grads.numel() >= self.grad_numel
        check(lib().cwdm_unet_backward(self._h, ctypes.c_void_p(packed.data_ptr()),
                                       ctypes.c_void_p(packed_bwd.data_ptr()), ctypes.c_void_p(x_ndhwc.data_ptr()),
                                       ctypes.c_void_p(t_f32.data_ptr()), ctypes.c_void_p(dout_ndhwc.data_ptr()),
                                       ctypes.c_void_p(grads.data_ptr()), B, D, H, W,
                                       ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(gws.data_ptr()),
                                       gws.numel(), seg_begin, seg_end, _stream()), "UNetModel.backward")
        return grads

    def backward_flops(self, B, D, H, W):
        return float(lib().cwdm_unet_backward_flops(self._h, B, D, H, W))

    def trace_tensors(self, ws, B, D, H, W):
        """Views of every block output left in the workspace (NDHWC)."""
        out = []
        n = lib().cwdm_unet_trace_count(self._h)
        off, ch, lv = ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()
        es = 4 if self.dtype == CWDM_F32 else 2
        for i in range(n):
            check(lib().cwdm_unet_trace_info(self._h, i, B, D, H, W, ctypes.byref(off), ctypes.byref(ch),
                                             ctypes.byref(lv)))
            if off.value < 0:
                out.append(None)
                continue
            d, h, w = D >> lv.value, H >> lv.value, W >> lv.value
            nbytes = B * d * h * w * ch.value * es
            buf = ws[off.value:off.value + nbytes].view(self.torch_dtype).view(B, d, h, w, ch.value)
            out.append(buf)
        return out

    def set_profiling(self, on):
        check(lib().cwdm_unet_set_profiling(self._h, 1 if on else 0))

    def profile_read(self):
        ms, fl, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        check(lib().cwdm_unet_profile_read(self._h, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(n)))
        return ms.value, fl.value, n.value
