"""TrainLoop (guided_diffusion/train_util.py:32-470) on the native U-Net.

Same constructor, ``run_loop`` / ``run_step`` / ``forward_backward`` /
``_anneal_lr`` / ``save_if_best`` contract.  What differs, MI355X-first:
  * backward: the native plan backward (UNetModel autograd Function), run in
    segments; with world_size > 1 a GradBucketReducer all-reduces finished
    gradient ranges (RCCL over xGMI) while later segments compute, and divides
    by the world size -- proper data parallelism (the reference never averages
    gradients across ranks: its sync_params is a no-op and it has no DDP);
  * optimizer: one fused AdamW launch over the flat parameter buffer
    (cwdm_hip.optim.FlatAdamW; torch.optim.AdamW semantics and state_dict);
  * norms / finiteness: 2 reductions over the flat buffers instead of ~760
    ``.item()`` syncs per step (:371-375);
  * logging goes to ``logger`` (wandb / TensorBoard are out of scope).
Checkpoints: ``brats_<contr>_BEST_<schedule>_<T>.pt`` (state_dict) and the
optimizer state under ``get_blob_logdir()/checkpoints`` (CWDM_LOGDIR, default
/data as in the reference, :499-504).
"""
import functools
import os
import time

import torch as th
import torch.distributed as dist

from . import dist_util, logger
from .resample import LossAwareSampler, UniformSampler
from .unet import UNetModel

INITIAL_LOG_LOSS_SCALE = 20.0


class TrainLoop:
    def __init__(self, *, model, diffusion, data, batch_size, in_channels, image_size, microbatch, lr, ema_rate,
                 log_interval, contr, save_interval, resume_checkpoint, resume_step, use_fp16=False,
                 fp16_scale_growth=1e-3, schedule_sampler=None, weight_decay=0.0, lr_anneal_steps=0,
                 dataset="brats", summary_writer=None, mode="default", loss_level="image",
                 sample_schedule="direct", diffusion_steps=1000):
        self.summary_writer = summary_writer
        self.mode = mode
        self.model = model
        self.diffusion = diffusion
        self.datal = data
        self.dataset = dataset
        self.iterdatal = iter(data)
        self.batch_size = batch_size
        self.in_channels = in_channels
        self.image_size = image_size
        self.contr = contr
        self.microbatch = microbatch if microbatch > 0 else batch_size
        self.lr = lr
        self.ema_rate = [ema_rate] if isinstance(ema_rate, float) else [float(x) for x in str(ema_rate).split(",")]
        self.log_interval = log_interval
        self.save_interval = save_interval
        self.resume_checkpoint = resume_checkpoint
        # use_fp16 enables dynamic loss scaling like the reference (amp.GradScaler,
        # train_util.py:84-87, :367-389, :457-458; there it scales an fp32 model).
        # A native model computing in fp16 (compute_dtype="fp16") needs it: the
        # MSE gradient of a 128^3 x 8 output is ~1e-7 per element, below fp16's
        # normal range, so it is scaled before the backward and unscaled (with
        # the non-finite check that skips the step) before AdamW
        self.use_fp16 = use_fp16
        fp16_compute = getattr(model, "compute_dtype", None) in ("fp16", "float16")
        self.grad_scaler = th.amp.GradScaler("cuda", enabled=bool(use_fp16 or fp16_compute) and th.cuda.is_available())
        # the loss-scaled optimizer step without GradScaler.step's found_inf read-back
        # (FlatAdamW skips on the device; env CWDM_SCALER_DEVICE_STEP=0: GradScaler.step)
        self.device_scaled_step = os.environ.get("CWDM_SCALER_DEVICE_STEP", "1") != "0"
        self.schedule_sampler = schedule_sampler or UniformSampler(diffusion)
        self.weight_decay = weight_decay
        self.lr_anneal_steps = lr_anneal_steps
        self.loss_level = loss_level
        self.step = 1
        self.resume_step = resume_step
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.global_batch = self.batch_size * self.world_size
        self.sync_cuda = th.cuda.is_available()
        self.sample_schedule = sample_schedule
        self.diffusion_steps = diffusion_steps
        self.best_losses = {}
        self.best_checkpoints = {}
        self.checkpoint_dir = os.path.join(get_blob_logdir(), "checkpoints")
        os.makedirs(self.checkpoint_dir, exist_ok=True)
        self._load_best_losses()
        self._load_and_sync_parameters()
        self.native = isinstance(model, UNetModel)
        if self.native:
            from cwdm_hip.ddp import GradBucketReducer
            from cwdm_hip.optim import FlatAdamW
            self.opt = FlatAdamW(self.model, lr=self.lr, weight_decay=self.weight_decay)
            self.reducer = GradBucketReducer() if self.world_size > 1 else None
            self.model._grad_hook = self.reducer
            # gradients land as views of the flat buffer straight in .grad
            # (FlatAdamW reads the flat buffer; autograd would clone each view)
            self.model.direct_grads = True
        else:
            self.opt = th.optim.AdamW(self.model.parameters(), lr=self.lr, weight_decay=self.weight_decay)
            self.reducer = None
        if self.resume_step:
            self._load_optimizer_state()
        self.last_info = {}

    # ---- checkpoints -------------------------------------------------------------
    def _load_best_losses(self):
        path = os.path.join(self.checkpoint_dir, "best_losses.txt")
        self.best_losses = {}
        if os.path.exists(path):
            try:
                with open(path) as f:
                    for line in f:
                        if line.strip():
                            k, v = line.strip().split(":")
                            self.best_losses[k] = float(v)
            except (OSError, ValueError) as e:
                print(f"Error loading best losses: {e}")
                self.best_losses = {}

    def _save_best_losses(self):
        with open(os.path.join(self.checkpoint_dir, "best_losses.txt"), "w") as f:
            for k, v in self.best_losses.items():
                f.write(f"{k}:{v}\n")

    def _load_and_sync_parameters(self):
        ckpt = find_resume_checkpoint() or self.resume_checkpoint
        if ckpt:
            self.resume_step = parse_resume_step_from_filename(ckpt)
            if not dist.is_initialized() or dist.get_rank() == 0:
                logger.log(f"loading model from checkpoint: {ckpt}...")
                self.model.load_state_dict(dist_util.load_state_dict(ckpt, map_location=dist_util.dev()))
        dist_util.sync_params(self.model.parameters())

    def _load_optimizer_state(self):
        ckpt = find_resume_checkpoint() or self.resume_checkpoint
        if not ckpt:
            return
        path = os.path.join(os.path.dirname(ckpt), f"opt{self.resume_step:06}.pt")
        if os.path.exists(path):
            logger.log(f"loading optimizer state from checkpoint: {path}")
            self.opt.load_state_dict(dist_util.load_state_dict(path, map_location=dist_util.dev()))
        else:
            print("no optimizer checkpoint exists")

    # ---- loop ------------------------------------------------------------------
    def _next_batch(self):
        try:
            return next(self.iterdatal)
        except StopIteration:
            self.iterdatal = iter(self.datal)
            return next(self.iterdatal)

    def run_loop(self):
        lossmse = None
        while not self.lr_anneal_steps or self.step + self.resume_step < self.lr_anneal_steps:
            batch = self._next_batch()
            cond = {}
            d = dist_util.dev()
            if self.mode == "i2i":
                batch = {k: (v.to(d) if th.is_tensor(v) else v) for k, v in batch.items()}
            else:
                batch = batch.to(d)
            t0 = time.time()
            lossmse, sample, sample_idwt = self.run_step(batch, cond)
            logger.logkv("time/step", time.time() - t0)
            if self.step % self.log_interval == 0:
                logger.logkv("loss/MSE", float(lossmse))
                logger.dumpkvs()
            if self.step % self.save_interval == 0:
                self.save_if_best(float(lossmse))
                if os.environ.get("DIFFUSION_TRAINING_TEST", "") and self.step > 0:
                    self.flush_finite_check()   # the last step's non-finite-loss warning still logs
                    return
            self.step += 1
        self.flush_finite_check()
        if lossmse is not None and (self.step - 1) % self.save_interval != 0:
            self.save_if_best(float(lossmse))

    def run_step(self, batch, cond, label=None, info=None):
        info = {} if info is None else info
        lossmse, sample, sample_idwt = self.forward_backward(batch, cond, label)
        if self.grad_scaler.is_enabled():
            self.grad_scaler.unscale_(self.opt)
        # native, no loss scaler: max |p| (before the update) and max |g| come out of the AdamW
        # pass itself (cwdm_adamw_maxabs), not two more passes over the 326 MB buffers
        # (env CWDM_FUSED_NORMS=0: the two separate reductions, A/B)
        fused_norms = (self.native and not self.grad_scaler.is_enabled() and hasattr(self.opt, "track_maxabs")
                       and os.environ.get("CWDM_FUSED_NORMS", "1") != "0")
        with th.no_grad():
            if fused_norms:
                self.opt.track_maxabs = True
            elif self.native:
                # max |p| over the flat buffers without a temporary (abs().max() wrote
                # a 326 MB |p| first: ~0.4 ms per step at 81.5 M parameters)
                inf = float("inf")
                info["norm/param_max"] = th.linalg.vector_norm(self.model.flat_params, inf)
                info["norm/grad_max"] = th.linalg.vector_norm(self.model.flat_grad(), inf)
            else:
                info["norm/param_max"] = max(p.abs().max() for p in self.model.parameters())
                info["norm/grad_max"] = max(p.grad.abs().max() for p in self.model.parameters() if p.grad is not None)
        self._check_finite(lossmse)
        if self.grad_scaler.is_enabled():
            found = self._scaler_found_inf() if self.device_scaled_step else None
            if found is not None:
                # sync-free: FlatAdamW skips on the device when found_inf is set
                # (GradScaler.step reads found_inf back first: the host waited for the
                # backward and the GPU for the host, ~1 ms per config-5 step)
                self.opt.step(found_inf=found)
            else:
                self.grad_scaler.step(self.opt)     # skipped when the unscaled gradients are not finite
            self.grad_scaler.update()
            # the scale tensor itself: get_scale() reads it back (.item()), a host
            # sync per step that the deferred finite check exists to avoid
            sc = getattr(self.grad_scaler, "_scale", None)
            info["scale"] = sc.detach().clone() if sc is not None else self.grad_scaler.get_scale()
        else:
            self.opt.step()
        if fused_norms:
            info["norm/param_max"] = self.opt.last_maxabs[0]
            info["norm/grad_max"] = self.opt.last_maxabs[1]
        self._anneal_lr()
        self.log_step()
        self.last_info = info
        return lossmse, sample, sample_idwt

    def _scaler_found_inf(self):
        """GradScaler's found_inf of this step (recorded by unscale_), for the
        optimizer's device-side skip; None where that does not apply (not the flat
        optimizer, several devices, or a torch whose GradScaler keeps it elsewhere)."""
        if not hasattr(self.opt, "_dstep"):
            return None
        try:
            st = self.grad_scaler._per_optimizer_states[id(self.opt)]
            vals = list(st["found_inf_per_device"].values())
        except (AttributeError, KeyError, TypeError):
            return None
        return vals[0] if len(vals) == 1 else None

    def _check_finite(self, lossmse):
        """The reference's per-step loss check (train_util.py run_step), read
        back one step late through pinned memory and an event so the host never
        waits for the device: the warning for step k is logged during step k+1
        (and by flush_finite_check)."""
        if not (lossmse.is_cuda and th.cuda.is_available()):
            if not th.isfinite(lossmse):
                logger.log(f"Model parameters are finite, but loss is not: {lossmse}", level=logger.WARN)
            return
        host = th.empty((), dtype=lossmse.dtype, pin_memory=True)
        host.copy_(lossmse.detach(), non_blocking=True)
        ev = th.cuda.Event()
        ev.record()
        pending = getattr(self, "_finite_pending", None)
        self._finite_pending = (host, ev)
        if pending is not None:
            self._report_finite(*pending)

    def _report_finite(self, host, ev):
        ev.synchronize()    # the previous step's loss: long done by now
        if not bool(th.isfinite(host)):
            logger.log(f"Model parameters are finite, but loss is not: {host}", level=logger.WARN)

    def flush_finite_check(self):
        pending = getattr(self, "_finite_pending", None)
        self._finite_pending = None
        if pending is not None:
            self._report_finite(*pending)

    def forward_backward(self, batch, cond, label=None):
        plist = self.model.param_list() if hasattr(self.model, "param_list") else self.model.parameters()
        for p in plist:
            p.grad = None
        batch_size = batch["t1n"].shape[0] if self.mode == "i2i" else batch.shape[0]
        t, weights = self.schedule_sampler.sample(batch_size, dist_util.dev())
        compute_losses = functools.partial(self.diffusion.training_losses, self.model, x_start=batch, t=t,
                                           model_kwargs=cond, labels=label, mode=self.mode, contr=self.contr)
        losses1 = compute_losses()
        losses, sample, sample_idwt = losses1
        if isinstance(self.schedule_sampler, LossAwareSampler):
            self.schedule_sampler.update_with_local_losses(t, losses["mse_wav"].detach().mean().expand(batch_size))
        loss = losses["mse_wav"].mean()   # equal channel weights (:442-449)
        lossmse = loss.detach()
        for key, values in losses.items():
            logger.logkv_mean(key, values.mean().detach())
        if self.grad_scaler.is_enabled():
            self.grad_scaler.scale(loss).backward()
        else:
            loss.backward()
        return lossmse, sample, sample_idwt

    def _anneal_lr(self):
        if not self.lr_anneal_steps:
            return
        frac_done = (self.step + self.resume_step) / self.lr_anneal_steps
        lr = self.lr * (1 - frac_done)
        for g in self.opt.param_groups:
            g["lr"] = lr

    def log_step(self):
        logger.logkv("step", self.step + self.resume_step)
        logger.logkv("samples", (self.step + self.resume_step + 1) * self.global_batch)

    def save_if_best(self, current_loss):
        modality = self.contr
        is_best = modality not in self.best_losses or current_loss < self.best_losses[modality]
        if not is_best:
            print(f"Loss {current_loss:.6f} not better than best {self.best_losses.get(modality, float('inf')):.6f} "
                  f"for {modality}")
            return
        self.best_losses[modality] = current_loss
        if dist.is_initialized() and dist.get_rank() != 0:
            return
        old = self.best_checkpoints.get(modality)
        if old and os.path.exists(old):
            os.remove(old)
        path = os.path.join(self.checkpoint_dir, f"brats_{modality}_BEST_{self.sample_schedule}_{self.diffusion_steps}.pt")
        th.save(self.model.state_dict(), path)
        self.best_checkpoints[modality] = path
        self._save_best_losses()
        th.save(self.opt.state_dict(), os.path.join(self.checkpoint_dir, f"opt_best_{modality}.pt"))


def parse_resume_step_from_filename(filename):
    """Trailing digits of the file stem (reference :486-506)."""
    split = os.path.basename(filename).split(".")[-2].split("_")[-1]
    digits = []
    for c in reversed(split):
        if not c.isdigit():
            break
        digits.append(c)
    s = "".join(reversed(digits))
    try:
        return int(s)
    except ValueError:
        return 0


def get_blob_logdir():
    return os.environ.get("CWDM_LOGDIR", "/data")


def find_resume_checkpoint():
    return None
