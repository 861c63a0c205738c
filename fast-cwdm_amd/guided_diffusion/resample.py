"""Timestep samplers (guided_diffusion/resample.py:7-154): t ~ U{0..T-1} via the
numpy global RNG, as the reference draws it (a14)."""
from abc import ABC, abstractmethod

import numpy as np
import torch as th
import torch.distributed as dist


def create_named_schedule_sampler(name, diffusion, maxt=None):
    if name == "uniform":
        return UniformSampler(diffusion, maxt)
    if name == "loss-second-moment":
        return LossSecondMomentResampler(diffusion)
    raise NotImplementedError(f"unknown schedule sampler: {name}")


def _upload(t, device):
    """Host -> device through pinned memory, asynchronous on the current stream."""
    if th.device(device).type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


class ScheduleSampler(ABC):
    @abstractmethod
    def weights(self):
        """Per-timestep sampling weights (positive, unnormalised)."""

    def sample(self, batch_size, device):
        w = self.weights()
        p = w / np.sum(w)
        indices_np = np.random.choice(len(p), size=(batch_size,), p=p)
        indices = _upload(th.from_numpy(indices_np).long(), device)
        # drawn in [0, T) on the host: training_losses need not read them back
        # from the device to range-check (no host/device sync per step)
        indices._cwdm_t_checked = len(p)
        weights_np = 1 / (len(p) * p[indices_np])
        weights = _upload(th.from_numpy(weights_np).float(), device)
        return indices, weights


class UniformSampler(ScheduleSampler):
    def __init__(self, diffusion, maxt=None):
        self.diffusion = diffusion
        self._weights = np.ones([maxt if maxt is not None else diffusion.num_timesteps])

    def weights(self):
        return self._weights


class LossAwareSampler(ScheduleSampler):
    def update_with_local_losses(self, local_ts, local_losses):
        ws = dist.get_world_size() if dist.is_initialized() else 1
        if ws == 1:
            self.update_with_all_losses([int(x) for x in local_ts.tolist()], [float(x) for x in local_losses.tolist()])
            return
        batch_sizes = [th.tensor([0], dtype=th.int32, device=local_ts.device) for _ in range(ws)]
        dist.all_gather(batch_sizes, th.tensor([len(local_ts)], dtype=th.int32, device=local_ts.device))
        batch_sizes = [x.item() for x in batch_sizes]
        max_bs = max(batch_sizes)
        timestep_batches = [th.zeros(max_bs).to(local_ts) for _ in batch_sizes]
        loss_batches = [th.zeros(max_bs).to(local_losses) for _ in batch_sizes]
        dist.all_gather(timestep_batches, local_ts)
        dist.all_gather(loss_batches, local_losses)
        timesteps = [x.item() for y, bs in zip(timestep_batches, batch_sizes) for x in y[:bs]]
        losses = [x.item() for y, bs in zip(loss_batches, batch_sizes) for x in y[:bs]]
        self.update_with_all_losses(timesteps, losses)

    @abstractmethod
    def update_with_all_losses(self, ts, losses):
        """Deterministic update from the gathered losses."""


class LossSecondMomentResampler(LossAwareSampler):
    def __init__(self, diffusion, history_per_term=10, uniform_prob=0.001):
        self.diffusion = diffusion
        self.history_per_term = history_per_term
        self.uniform_prob = uniform_prob
        self._loss_history = np.zeros([diffusion.num_timesteps, history_per_term], dtype=np.float64)
        self._loss_counts = np.zeros([diffusion.num_timesteps], dtype=np.int64)

    def weights(self):
        if not self._warmed_up():
            return np.ones([self.diffusion.num_timesteps], dtype=np.float64)
        weights = np.sqrt(np.mean(self._loss_history ** 2, axis=-1))
        weights /= np.sum(weights)
        weights *= 1 - self.uniform_prob
        weights += self.uniform_prob / len(weights)
        return weights

    def update_with_all_losses(self, ts, losses):
        for t, loss in zip(ts, losses):
            if self._loss_counts[t] == self.history_per_term:
                self._loss_history[t, :-1] = self._loss_history[t, 1:]
                self._loss_history[t, -1] = loss
            else:
                self._loss_history[t, self._loss_counts[t]] = loss
                self._loss_counts[t] += 1

    def _warmed_up(self):
        return (self._loss_counts == self.history_per_term).all()
