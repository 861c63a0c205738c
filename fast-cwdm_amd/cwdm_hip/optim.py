"""Fused AdamW over a flat parameter buffer (replaces torch.optim.AdamW at
guided_diffusion/train_util.py:111 for the native UNetModel).

The native UNetModel keeps every parameter as a view of one contiguous fp32
buffer (state_dict order) and its backward writes one contiguous gradient
buffer, so the whole optimizer step is ONE launch of ``cwdm_adamw`` over
81.5 M elements instead of ~760 per-tensor kernels.  Semantics, hyper-
parameters, ``param_groups[0]["lr"]`` (annealed by TrainLoop._anneal_lr) and
``state_dict()`` layout are torch.optim.AdamW's, so optimizer checkpoints stay
interchangeable with the reference's.
"""
import os

import torch

from ._lib import check, lib
from .ops import _need_cuda, _stream


# env CWDM_PER_PARAM_STEP=1: a fresh step tensor per parameter each step (the old host cost, A/B knob)
_PER_PARAM_STEP = os.environ.get("CWDM_PER_PARAM_STEP", "0") == "1"


class FlatAdamW(torch.optim.Optimizer):
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, direct_grads=False):
        params = list(model.parameters())
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        flat = model.flat_params
        _need_cuda(flat)
        o = 0
        for p in params:
            if p.data_ptr() != flat.data_ptr() + 4 * o or p.dtype != torch.float32:
                raise ValueError("FlatAdamW: parameters must be in-order views of the model's flat fp32 buffer")
            o += p.numel()
        if o != flat.numel():
            raise ValueError("FlatAdamW: flat buffer / parameter size mismatch")
        self._model = model
        # direct_grads=True: the model's backward hands its flat gradient buffer
        # over as the parameters' .grad views (no per-parameter copies; flat_grad()
        # is that buffer).  Opt-in, since it changes what torch.autograd.grad and
        # backward(inputs=...) see on that model; TrainLoop sets model.direct_grads
        # itself.  Either way step() reads model.flat_grad().
        if direct_grads:
            model.direct_grads = True
        self._flat = flat
        self._m = torch.zeros_like(flat)
        self._v = torch.zeros_like(flat)
        self._step = 0
        self._dstep = None   # device step count once a found_inf step ran (sync-free loss scaling)
        self._fi_keep = None
        # track_maxabs: step() also leaves last_maxabs = [max |p| before the update, max |g|]
        # (a fresh 2-element device tensor per step, cwdm_adamw_maxabs: the same pass)
        self.track_maxabs = False
        self.last_maxabs = None
        self._bind_state()

    def _bind_state(self):
        # one step tensor shared by every parameter's state (torch keeps one per
        # parameter: 230 host fill_ calls per step, ~0.5 ms of host time while the
        # next step waited to launch); state_dict() hands each entry the same value
        self._step_t = torch.tensor(float(self._step))
        o = 0
        for p in self.param_groups[0]["params"]:
            n = p.numel()
            self.state[p] = {"step": self._step_t,
                             "exp_avg": self._m[o:o + n].view_as(p),
                             "exp_avg_sq": self._v[o:o + n].view_as(p)}
            o += n

    @torch.no_grad()
    def step(self, closure=None, found_inf=None):
        """found_inf (device tensor, GradScaler's after unscale_): the sync-free
        loss-scaled step -- the update is skipped on the device when it is
        non-zero (GradScaler.step would read it back first and skip the call), and
        from then on the step count lives on the device (state_dict() reads it)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self._model.flat_grad()
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        if found_inf is not None or self._dstep is not None:
            if self._dstep is None:
                self._dstep = torch.tensor(float(self._step), dtype=torch.float64, device=self._flat.device)
            fi = found_inf.reshape(-1)[:1].float().contiguous() if found_inf is not None else None
            check(lib().cwdm_adamw_device_step(self._flat.data_ptr(), g.data_ptr(), self._m.data_ptr(), self._v.data_ptr(),
                                               self._flat.numel(), float(grp["lr"]), float(b1), float(b2),
                                               float(grp["eps"]), float(grp["weight_decay"]), self._dstep.data_ptr(),
                                               fi.data_ptr() if fi is not None else None, _stream()), "AdamW.step")
            self._fi_keep = fi   # (alive until the launch has read it)
            torch.autograd.graph.increment_version(self._flat)
            self._model.mark_params_changed()
            return loss
        self._step += 1
        args = (self._flat.data_ptr(), g.data_ptr(), self._m.data_ptr(), self._v.data_ptr(), self._flat.numel(),
                float(grp["lr"]), float(b1), float(b2), float(grp["eps"]), float(grp["weight_decay"]), self._step)
        if self.track_maxabs:
            self.last_maxabs = torch.empty(2, dtype=torch.float32, device=self._flat.device)
            check(lib().cwdm_adamw_maxabs(*args, self.last_maxabs.data_ptr(), _stream()), "AdamW.step")
        else:
            check(lib().cwdm_adamw(*args, _stream()), "AdamW.step")
        # the kernel wrote through raw pointers: the model must re-pack its
        # kernel-layout weights (the parameters' own version counters do not
        # see writes to the flat buffer)
        torch.autograd.graph.increment_version(self._flat)
        self._model.mark_params_changed()
        if _PER_PARAM_STEP:
            for st in self.state.values():
                st["step"] = torch.tensor(float(self._step))
        else:
            self._step_t.fill_(float(self._step))
        return loss

    def state_dict(self):
        # per-parameter step tensors in the saved form, as torch.optim.AdamW keeps them
        # (a shared one loaded into torch's AdamW would be incremented once per parameter)
        if self._dstep is not None:   # the device count (skipped steps not counted): one read-back here
            self._step = int(self._dstep.item())
            self._step_t.fill_(float(self._step))
        sd = super().state_dict()
        sd["state"] = {k: {**v, "step": v["step"].clone()} if "step" in v else v for k, v in sd["state"].items()}
        return sd

    def zero_grad(self, set_to_none=True):
        for p in self.param_groups[0]["params"]:
            p.grad = None

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        o = 0
        step = 0
        for p in self.param_groups[0]["params"]:
            n = p.numel()
            st = self.state.get(p, {})
            if "exp_avg" in st:
                self._m[o:o + n].copy_(st["exp_avg"].reshape(-1))
                self._v[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                step = int(float(st["step"]))
            o += n
        self._step = step
        self._dstep = None
        self._bind_state()
