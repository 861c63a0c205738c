"""Timestep respacing (drop-in for guided_diffusion/respace.py:7-132).

``_WrappedModel`` keeps the reference contract (spaced t -> original t via
``timestep_map``), but the map lives on the device once instead of being
re-uploaded per call (:127-132), and the native sampling loop reads the mapped
value on the host so no per-step H2D copy or sync remains.
"""
import os

import numpy as np
import torch as th

from .gaussian_diffusion import GaussianDiffusion


def space_timesteps(num_timesteps, section_counts):
    if isinstance(section_counts, str):
        if section_counts.startswith("ddim"):
            desired_count = int(section_counts[len("ddim"):])
            for i in range(1, num_timesteps):
                if len(range(0, num_timesteps, i)) == desired_count:
                    return set(range(0, num_timesteps, i))
            raise ValueError(f"cannot create exactly {num_timesteps} steps with an integer stride")
        section_counts = [int(x) for x in section_counts.split(",")]
    size_per = num_timesteps // len(section_counts)
    extra = num_timesteps % len(section_counts)
    start_idx = 0
    all_steps = []
    for i, section_count in enumerate(section_counts):
        size = size_per + (1 if i < extra else 0)
        if size < section_count:
            raise ValueError(f"cannot divide section of {size} steps into {section_count}")
        frac_stride = 1 if section_count <= 1 else (size - 1) / (section_count - 1)
        cur_idx = 0.0
        taken = []
        for _ in range(section_count):
            taken.append(start_idx + round(cur_idx))
            cur_idx += frac_stride
        all_steps += taken
        start_idx += size
    return set(all_steps)


# env CWDM_TSMAP_SHARED=0: a device timestep map per wrapper (the old per-step copy, A/B knob)
_SHARED_TS_MAP = os.environ.get("CWDM_TSMAP_SHARED", "1") != "0"

class SpacedDiffusion(GaussianDiffusion):
    def __init__(self, use_timesteps, **kwargs):
        self.use_timesteps = set(use_timesteps)
        self.timestep_map = []
        self.original_num_steps = len(kwargs["betas"])
        base = GaussianDiffusion(**kwargs)
        last_alpha_cumprod = 1.0
        new_betas = []
        # the base (shared) schedule; FATS per-band tables are rebuilt from it by
        # GaussianDiffusion (each band's acp_k is a function of acp at the same step)
        for i, alpha_cumprod in enumerate(base.base_alphas_cumprod):
            if i in self.use_timesteps:
                new_betas.append(1 - alpha_cumprod / last_alpha_cumprod)
                last_alpha_cumprod = alpha_cumprod
                self.timestep_map.append(i)
        kwargs["betas"] = np.array(new_betas)
        super().__init__(**kwargs)

    def p_mean_variance(self, model, *args, **kwargs):
        return super().p_mean_variance(self._wrap_model(model), *args, **kwargs)

    def p_sample(self, model, *args, **kwargs):
        return super().p_sample(self._wrap_model(model), *args, **kwargs)

    def training_losses(self, model, *args, **kwargs):
        return super().training_losses(self._wrap_model(model), *args, **kwargs)

    def ddim_sample(self, model, *args, **kwargs):
        # the reference's ddim_sample reaches the model through the wrapped
        # p_mean_variance (:90-93); this one calls the model itself
        return super().ddim_sample(self._wrap_model(model), *args, **kwargs)

    def _wrap_model(self, model):
        if isinstance(model, _WrappedModel):
            return model
        # the device copy of timestep_map is shared by every wrapper of this diffusion:
        # training_losses wraps the model on every step, and a fresh th.tensor(list,
        # device=cuda) per wrapper is a pageable host->device copy that waits for the
        # whole queue (the config-5 training step spent ~6 ms of host time blocked there)
        maps = self.__dict__.setdefault("_ts_maps", {}) if _SHARED_TS_MAP else None
        return _WrappedModel(model, self.timestep_map, self.rescale_timesteps, self.original_num_steps, maps)

    def _scale_timesteps(self, t):
        return t  # scaling is done by the wrapped model

    def _model_timestep(self, i):
        v = float(self.timestep_map[i])
        if self.rescale_timesteps:
            v = v * (1000.0 / self.original_num_steps)
        return v


class _WrappedModel:
    def __init__(self, model, timestep_map, rescale_timesteps, original_num_steps, maps=None):
        self.model = model
        self.timestep_map = timestep_map
        self.rescale_timesteps = rescale_timesteps
        self.original_num_steps = original_num_steps
        self._maps = maps if maps is not None else {}

    def parameters(self):
        return self.model.parameters()

    def __call__(self, x, ts, **kwargs):
        key = (str(ts.device), ts.dtype)
        if key not in self._maps:
            self._maps[key] = th.tensor(self.timestep_map, device=ts.device, dtype=ts.dtype)
        new_ts = self._maps[key][ts]
        if self.rescale_timesteps:
            new_ts = new_ts.float() * (1000.0 / self.original_num_steps)
        return self.model(x, new_ts, **kwargs)
