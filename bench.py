"""Benchmark: denoising-steps/s on 8-channel 128^3 wavelet volumes (BASELINE.json
config 2: BraTS 4-modality -> 1 conditional synthesis, 1000-step DDPM, bf16).

One step = one p_sample of the i2i wavelet diffusion: the production U-Net
(run.sh configuration, 81.5 M parameters, seeded non-zero weights) on
[x_t (8) | cond (24)] at 128^3 subbands, then the fused IDWT->clamp->DWT ->
posterior-mean -> +sigma*noise epilogue, noise drawn with th.randn_like like the
reference.  Inputs are synthetic 256^3 phantoms (no datasets offline), DWT'd on
the GPU before the timed region.

Multi-GPU: sampling shards by volume ("replicas only"): each rank
denoises its own volume, no collective on the data path; value = all ranks'
steps / max-over-ranks time.  `--gpus N` without torchrun's environment
launches the N ranks itself (fresh child processes, started before this
process touches the GPU).  The config-3 side figure `train_ddp` is the one
leg with a real exchange: TrainLoop.run_step at 128^3 bf16, batch 1 per GPU,
the bucketed gradient all-reduce over RCCL overlapped with the backward.

Prints ONE JSON line on rank 0 (contract in the task statement), including
`roofline` for the dominant kernel (conv3d implicit GEMM, all launches of a
step) and `cpu_baseline` (the CPU oracle timed on this host, rank 0, N=1).
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "fast-cwdm_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

TRAFFIC_JSONS = [os.path.join(ROOT, "profiles", r, "pmc_traffic.json") for r in ("r06", "r05", "r04", "r03", "r02", "r01")]
BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
F32_PEAK_TFLOPS = 157.3


def seeded_weights(model, seed):
    """Non-degenerate weights of the production architecture (the reference's
    zero-init would make every ResBlock an identity)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if p.dim() == 1 and (".in_layers.0." in name or ".out_layers.0." in name or name.startswith("out.0.")):
                p.copy_((1.0 if name.endswith("weight") else 0.0) + 0.1 * torch.randn(p.shape, generator=g))
            elif p.dim() >= 2:
                p.copy_(torch.randn(p.shape, generator=g) / math.sqrt(p[0].numel()))
            else:
                p.copy_(0.05 * torch.randn(p.shape, generator=g))


def phantom_gpu(n, seed, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    ax = (0.75 + 0.15 * torch.rand(3, generator=g)).tolist()
    lin = torch.linspace(-1, 1, n, device=device)
    z, y, x = lin.view(n, 1, 1), lin.view(1, n, 1), lin.view(1, 1, n)
    mask = (z / ax[0]) ** 2 + (y / ax[1]) ** 2 + (x / ax[2]) ** 2 <= 1.0
    img = torch.zeros(n, n, n, device=device)
    for _ in range(6):
        c = ((torch.rand(3, generator=g) - 0.5) * 1.2).tolist()
        s = float(0.15 + 0.35 * torch.rand(1, generator=g))
        a = float(0.3 + 0.7 * torch.rand(1, generator=g))
        img += a * torch.exp(-((z - c[0]) ** 2 + (y - c[1]) ** 2 + (x - c[2]) ** 2) / (2 * s * s))
    img = img * mask
    return (img / img.max()).clamp(0, 1).view(1, 1, n, n, n)


def build(args, device):
    from guided_diffusion import script_util
    margs = script_util.run_sh_model_args(diffusion_steps=1000, sample_schedule="direct")
    keys = script_util.model_and_diffusion_defaults().keys()
    model, diffusion = script_util.create_model_and_diffusion(**{k: margs[k] for k in keys},
                                                              compute_dtype=args.dtype)
    diffusion.mode = "i2i"
    seeded_weights(model, 1)
    model.to(device)
    return model, diffusion


def cpu_threads():
    """Host cores this process may use: its CPU affinity, capped by a cgroup
    CPU quota when one is set (the GPU box's share of a larger machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(state, cond, x_T, threads, T=1000, warmup=1, steps=2):
    """the oracle (PyTorch-CPU fp32 restatement of the
    reference path) on this host with the GPU leg's own inputs -- the same
    seeded weights (state_dict of the benchmarked model), phantom cond and x_T
    -- 1 warm-up step (t = T-1) then 2 timed steps (t = T-2, T-3)."""
    from oracle import diffusion as od, unet as ou
    torch.set_num_threads(threads)
    tab = od.Tables(od.beta_schedule("linear", T, "direct"))
    model = ou.OracleUNet(state)
    g = torch.Generator().manual_seed(7)
    x = x_T
    dts = []
    with torch.no_grad():
        for k in range(warmup + steps):
            t = torch.tensor([T - 1 - k])
            noise = torch.randn(x.shape, generator=g)
            t0 = time.perf_counter()
            x = od.p_sample(tab, model, x, t, cond, noise)["sample"]
            dts.append(time.perf_counter() - t0)
    return dts[warmup:]


def cpu_config1(threads):
    """BASELINE.md §3 / config 1 end to end on CPU: the 64^3 phantom set ->
    Haar DWT conditioning -> 2-step 'sampled' p_sample_loop with the tiny U-Net
    (seeded non-zero weights) -> IDWT, clamp, brain mask (oracle.cases.c1_run),
    wall clock of one full run after one warm-up run."""
    from oracle import cases
    torch.set_num_threads(threads)
    cases.c1_run()
    t0 = time.perf_counter()
    cases.c1_run()
    return time.perf_counter() - t0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """`--gpus N` outside torchrun: start N fresh rank processes (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_* set) and return the worst exit code.
    This process never touches the GPU and never execs."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def time_loop(loop, n, world, sync):
    for _ in range(n[0]):
        next(loop)
    sync()
    t0 = time.perf_counter()
    for _ in range(n[1]):
        next(loop)
    sync()
    return time.perf_counter() - t0


def train_leg(model, diffusion, n, rank, world, device, steps, warmup, sync, max_over_ranks):
    """Config 3: TrainLoop.run_step (4 Haar DWTs + q_sample into the 32-channel
    input, native forward, MSE, segmented native backward with the bucketed
    gradient all-reduce over RCCL overlapped, fused AdamW), batch 1 per GPU."""
    import numpy as np
    from guided_diffusion import train_util
    os.environ.setdefault("CWDM_LOGDIR", os.path.join(ROOT, "gpurun_out", "bench_train"))
    np.random.seed(3)
    n2 = 2 * n
    batch = {k: phantom_gpu(n2, 1000 + 100 * rank + j, device) for j, k in enumerate(("t1n", "t1c", "t2w", "t2f"))}
    loop = train_util.TrainLoop(model=model, diffusion=diffusion, data=[batch], batch_size=1, in_channels=32,
                                image_size=n2, microbatch=-1, lr=1e-5, ema_rate="0.9999", log_interval=10 ** 9,
                                contr="t1n", save_interval=10 ** 9, resume_checkpoint="", resume_step=0,
                                mode="i2i", diffusion_steps=1000)
    for _ in range(warmup):
        loop.run_step(batch, {})
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss, _, _ = loop.run_step(batch, {})
    sync()
    dt = max_over_ranks(time.perf_counter() - t0)
    plan = model.plan
    fl = plan.flops(1, n, n, n) + plan.backward_flops(1, n, n, n)
    per = dt / steps
    return {"workload": "config3: TrainLoop.run_step, 128^3 subbands (256^3 phantoms x 4 modalities), batch 1 per GPU, "
                        f"{model.compute_dtype}, bucketed gradient all-reduce "
                        f"({'RCCL' if world > 1 and dist.get_backend() == 'nccl' else dist.get_backend() if world > 1 else 'none'})"
                        " overlapped with the segmented native backward, fused AdamW",
            "volumes_per_s": round(world * steps / dt, 4), "ms_per_step": round(1000 * per, 2), "steps": steps,
            "warmup": warmup, "n_gpus": world, "conv_tflop_per_step": round(fl / 1e12, 2),
            "mfma_frac": round(fl / per / 1e12 / BF16_PEAK_TFLOPS, 4), "loss": round(float(loss), 6),
            "scaling": "weak"}


def config5_leg(args, device, rank, world, sync, max_over_ranks):
    """Config 5 (spec-only): 224^3 phantoms -> 2-level block
    wavelet analysis (56^3 x 64 channels per modality, straight from the GPU
    kernel) -> 3-level U-Net (256 -> 64 channels, mc 64, mult 1,2,2) -> the
    2-level fused sampler step with FATS per-subband schedules (shifts from
    the conditioning's subband energies), HIP-graph-captured loop, bf16."""
    from cwdm_hip import ops
    from guided_diffusion import fats, script_util
    n = 224
    g = n // 4
    model = script_util.create_model(image_size=n, num_channels=64, num_res_blocks=2, channel_mult="1,2,2",
                                     attention_resolutions="", dims=3, num_groups=32, in_channels=256,
                                     out_channels=64, bottleneck_attention=False, resample_2d=False,
                                     resblock_updown=True, compute_dtype=args.config5_dtype)
    seeded_weights(model, 5)
    model.to(device)
    t0 = time.perf_counter()
    cond_cl = torch.empty(1, g, g, g, 192, device=device)
    for k in range(3):
        ops.wavelet2_analysis(phantom_gpu(n, 500 + 10 * rank + k, device), out=cond_cl, c0=64 * k)
    sync()
    t_front = time.perf_counter() - t0
    cond = cond_cl.permute(0, 4, 1, 2, 3)
    shifts = fats.band_log_snr_shifts(
        fats.subband_energy(cond[:, :64], levels=2) + fats.subband_energy(cond[:, 64:128], levels=2))
    diffusion = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                      band_log_snr_shift=shifts, wavelet_levels=2)
    torch.manual_seed(4321 + rank)
    x_T = torch.randn(1, 64, g, g, g, device=device)
    K = args.config5
    loop = diffusion._native_loop(model, x_T, list(range(1000))[::-1][:K + 4], cond.contiguous(), True,
                                  graph=bool(args.graph), fresh_outputs=False, need_pred=False)
    dt = max_over_ranks(time_loop(loop, (3, K), world, sync))
    loop.close()
    per = dt / K
    fl = model.plan.flops(1, g, g, g)
    res = {"workload": "config5: 224^3 input, 2-level block wavelet (56^3 x 64 ch per modality, 15 subbands), "
                       "FATS per-subband schedules, 3-level U-Net (256->64 ch, mc 64, mult 1,2,2, 2 res blocks), "
                       f"{args.config5_dtype}, {'HIP-graph' if args.graph else 'eager'} loop, one volume per GPU",
           "denoising_steps_per_s": round(world * K / dt, 3), "ms_per_step": round(1000 * per, 3), "steps": K,
           "s_per_volume": {"1000_steps": round(1000 * per, 2), "50_steps": round(50 * per, 3)},
           "front_end_ms": round(1000 * t_front, 2), "unet_tflop_per_step": round(fl / 1e12, 3),
           "mfma_frac": round(fl / per / 1e12 / BF16_PEAK_TFLOPS, 4), "dtype": args.config5_dtype}
    del model, loop
    torch.cuda.empty_cache()
    return res


def train5_leg(args, device, rank, world, sync, max_over_ranks):
    """Config 5 training: TrainLoop.run_step on the 2-level representation
    (224^3 phantoms x 4 modalities -> cwdm_prepare_batch2 -> the config-5
    3-level U-Net, FATS per-channel q_sample rows -> segmented native backward
    (+ RCCL bucketed all-reduce when N > 1) -> fused AdamW), batch 1 per GPU, in --config5-dtype
    (fp16: dynamic loss scaling, TrainLoop's GradScaler)."""
    import numpy as np
    from cwdm_hip import ops
    from guided_diffusion import fats, script_util, train_util
    os.environ.setdefault("CWDM_LOGDIR", os.path.join(ROOT, "gpurun_out", "bench_train5"))
    n, g = 224, 56
    model = script_util.create_model(image_size=n, num_channels=64, num_res_blocks=2, channel_mult="1,2,2",
                                     attention_resolutions="", dims=3, num_groups=32, in_channels=256,
                                     out_channels=64, bottleneck_attention=False, resample_2d=False,
                                     resblock_updown=True, compute_dtype=args.config5_dtype)
    seeded_weights(model, 5)
    model.to(device)
    batch = {k: phantom_gpu(n, 700 + 100 * rank + j, device) for j, k in enumerate(("t1n", "t1c", "t2w", "t2f"))}
    e = sum(fats.subband_energy(ops.wavelet2_analysis(batch[k]).permute(0, 4, 1, 2, 3), levels=2)
            for k in ("t1c", "t2w"))
    diffusion = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                      band_log_snr_shift=fats.band_log_snr_shifts(e),
                                                      wavelet_levels=2)
    np.random.seed(5)
    loop = train_util.TrainLoop(model=model, diffusion=diffusion, data=[batch], batch_size=1, in_channels=256,
                                image_size=n, microbatch=-1, lr=1e-5, ema_rate="0.9999", log_interval=10 ** 9,
                                contr="t1n", save_interval=10 ** 9, resume_checkpoint="", resume_step=0,
                                mode="i2i", diffusion_steps=1000)
    for _ in range(2):
        loop.run_step(batch, {})
    sync()
    K = args.train5
    t0 = time.perf_counter()
    for _ in range(K):
        loss, _, _ = loop.run_step(batch, {})
    sync()
    dt = max_over_ranks(time.perf_counter() - t0)
    fl = model.plan.flops(1, g, g, g) + model.plan.backward_flops(1, g, g, g)
    per = dt / K
    res = {"workload": "config5 training: TrainLoop.run_step, 224^3 phantoms x 4 modalities -> 2-level block "
                       "wavelets (56^3 x 64 ch per modality), FATS per-channel q_sample, 3-level U-Net (256->64 ch), "
                       f"{args.config5_dtype}{' (dynamic loss scaling)' if loop.grad_scaler.is_enabled() else ''}, "
                       "batch 1 per GPU, gradient all-reduce "
                       f"({'RCCL' if world > 1 and dist.get_backend() == 'nccl' else dist.get_backend() if world > 1 else 'none'})",
           "volumes_per_s": round(world * K / dt, 4), "ms_per_step": round(1000 * per, 2), "steps": K,
           "conv_tflop_per_step": round(fl / 1e12, 3), "mfma_frac": round(fl / per / 1e12 / BF16_PEAK_TFLOPS, 4),
           "loss": round(float(loss), 6), "scaling": "weak", "dtype": args.config5_dtype}
    if loop.grad_scaler.is_enabled():
        res["loss_scale"] = float(loop.grad_scaler.get_scale())
    del model, loop
    torch.cuda.empty_cache()
    return res


def wavunet_leg(args, diffusion, x_T, cond, device, world, sync, max_over_ranks):
    """f4: the frequency-aware WavUNetModel (use_freq=True, script_util's
    configuration at the run.sh sizes: mc 64, mult 1,2,2,4,4, 2 res blocks,
    90.1 M parameters) in the same 128^3 sampling loop (HIP graph, bf16)."""
    from guided_diffusion import script_util
    n = x_T.shape[-1]
    model = script_util.create_model(image_size=2 * n, num_channels=64, num_res_blocks=2, channel_mult="1,2,2,4,4",
                                     attention_resolutions="", dims=3, num_groups=32, in_channels=32,
                                     out_channels=8, bottleneck_attention=False, resblock_updown=True,
                                     use_freq=True, compute_dtype=args.dtype)
    seeded_weights(model, 9)
    model.to(device)
    K = args.wavunet
    loop = diffusion._native_loop(model, x_T, list(range(diffusion.num_timesteps))[::-1][:K + 4], cond, True,
                                  graph=bool(args.graph), fresh_outputs=False, need_pred=False)
    dt = max_over_ranks(time_loop(loop, (3, K), world, sync))
    loop.close()
    per = dt / K
    fl = model.plan.flops(1, n, n, n)
    res = {"workload": f"f4: WavUNetModel (use_freq, mc 64, mult 1,2,2,4,4, 2 res blocks, "
                       f"{sum(p.numel() for p in model.parameters()) / 1e6:.1f}M params), {n}^3 subbands, {args.dtype}, "
                       f"{'HIP-graph' if args.graph else 'eager'} 1000-step DDPM loop, one volume per GPU",
           "denoising_steps_per_s": round(world * K / dt, 3), "ms_per_step": round(1000 * per, 3), "steps": K,
           "unet_tflop_per_step": round(fl / 1e12, 3), "mfma_frac": round(fl / per / 1e12 / BF16_PEAK_TFLOPS, 4)}
    del model, loop
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grid", type=int, default=128, help="subband edge (image edge = 2x)")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--graph", type=int, default=1, help="replay one HIP-graph-captured step per timestep")
    ap.add_argument("--respaced", type=int, default=1,
                    help="also time config 4: a full 50-step respaced DDIM (ddim50) volume, graph-captured loop")
    ap.add_argument("--batched", type=int, default=2,
                    help="also time B volumes denoised together in one batched step (serving throughput; "
                         "0 = skip); reported beside, never as, the B=1 metric")
    ap.add_argument("--fp32", type=int, default=3, help="also time K steps of the fp32 parity mode (0 = skip)")
    ap.add_argument("--fp32x", type=int, default=5, help="also time K steps of the accurate fast mode (fp32 storage, "
                                                        "split-bf16 conv MFMAs; 0 = skip)")
    ap.add_argument("--train", type=int, default=5, help="config-3 train_ddp side figure: timed steps (0 = skip)")
    ap.add_argument("--wavunet", type=int, default=10, help="f4 side figure: WavUNetModel at 128^3, timed steps "
                                                            "(0 = skip)")
    ap.add_argument("--config5", type=int, default=10, help="config-5 side figure (224^3, 2-level wavelets + FATS): "
                                                            "timed steps (0 = skip)")
    ap.add_argument("--train5", type=int, default=3, help="config-5 training side figure (224^3, 2-level "
                                                          "wavelets + FATS): timed steps (0 = skip)")
    ap.add_argument("--config5-dtype", default="fp16", help="compute dtype of the config-5 legs (BASELINE.json "
                                                            "config 5: fp16)")
    ap.add_argument("--fp16", type=int, default=5, help="also time K config-2 steps with the U-Net in fp16 "
                                                        "(0 = skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the rank launch / barrier / max-over-ranks plumbing only")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CWDM_BENCH_REHEARSE=1: every rank on cuda:0 with gloo (a 1-GPU rehearsal
    # of the N-rank code path; the driver's N-GPU runs use RCCL, one GPU per rank)
    rehearse = os.environ.get("CWDM_BENCH_REHEARSE") == "1" or args.dry_run
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            # one GPU per rank, bound at init (RCCL communicator on cuda:LOCAL_RANK)
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.dry_run:
        def mor(v):
            tt = torch.tensor([v], dtype=torch.float64)
            if world > 1:
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            return float(tt)
        if world > 1:
            dist.barrier()
        v = mor(float(rank))
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "max_rank": v,
                              "backend": dist.get_backend() if world > 1 else None}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)

    def max_over_ranks(v):
        if world == 1:
            return v
        tt = torch.tensor([v], dtype=torch.float64, device="cpu" if rehearse else device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    model, diffusion = build(args, device)
    n = args.grid
    # synthetic conditioning: 3 phantoms at (2n)^3 -> Haar DWT (LLL/3) on the GPU
    from cwdm_hip import ops
    cond = torch.empty(1, 24, n, n, n, device=device)
    V = n ** 3
    for k in range(3):
        vol = phantom_gpu(2 * n, 100 + 10 * rank + k, device)
        ops.dwt3d(vol, lll_div3=True, out=cond[:, 8 * k:], out_strides=(V, 24 * V, 0, 1))
    torch.manual_seed(1234 + rank)
    x_T = torch.randn(1, 8, n, n, n, device=device)
    T = diffusion.num_timesteps
    total = args.warmup + args.steps
    assert total <= T
    loop = diffusion._native_loop(model, x_T, list(range(T))[::-1][:total + 2], cond, True,
                                  graph=bool(args.graph), fresh_outputs=False, need_pred=False)
    for _ in range(args.warmup):
        next(loop)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        next(loop)
    sync()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    loop.close()
    ops.check_device_status("bench timed loop")   # (after the timed region: it synchronises)

    # roofline of the dominant kernel -- the implicit-GEMM MFMA conv kernels:
    # hipEvents around each of their launches over one extra (eager) step, on
    # the stream they run on; GroupNorm pre-passes, split-K finishes and the
    # sampler are HBM-bound kernels outside this figure
    plan = model.plan
    plan.set_profiling(True)
    loop = diffusion._native_loop(model, x_T, [T - 1], cond, True, graph=False)
    next(loop)
    torch.cuda.synchronize()
    conv_ms, conv_flops, n_conv = plan.profile_read()
    plan.set_profiling(False)
    loop.close()
    step_flops = plan.flops(1, n, n, n)

    # serving side-figure: B volumes per batched step (the 16^3 / 8^3 levels of
    # a single volume leave the chip idle; a batch fills them)
    batched = None
    if args.batched > 1:
        Bv = args.batched
        xb = x_T.expand(Bv, -1, -1, -1, -1).contiguous()
        cb = cond.expand(Bv, -1, -1, -1, -1).contiguous()
        nb = 6
        lb = diffusion._native_loop(model, xb, list(range(T))[::-1][:nb + 3], cb, True, graph=bool(args.graph),
                                    fresh_outputs=False, need_pred=False)
        tb = max_over_ranks(time_loop(lb, (2, nb), world, sync))
        lb.close()
        batched = {"batch_per_gpu": Bv, "ms_per_batched_step": round(1000 * tb / nb, 3),
                   "volume_steps_per_s": round(world * Bv * nb / tb, 3)}
        del xb, cb
        torch.cuda.empty_cache()

    # config 4: respaced 50-step DDIM sampling of one whole volume (timestep_respacing
    # "ddim50" = stride-20 subset of the 1000-step schedule; i2i DDIM update in the
    # fused sampler kernel), graph-captured loop
    respaced = None
    if args.respaced:
        from guided_diffusion import respace
        sp = respace.SpacedDiffusion(use_timesteps=respace.space_timesteps(1000, "ddim50"),
                                     betas=diffusion.betas, model_mean_type=diffusion.model_mean_type,
                                     model_var_type=diffusion.model_var_type, loss_type=diffusion.loss_type,
                                     rescale_timesteps=diffusion.rescale_timesteps)
        sp.mode = "i2i"
        sp.use_hip_graph = bool(args.graph)
        for rep in range(2):   # first pass warms the graph capture path
            sync()
            t1 = time.perf_counter()
            sp.ddim_sample_loop(model, tuple(x_T.shape), noise=x_T, cond=cond, eta=0.0)
            sync()
            rs = time.perf_counter() - t1
        rs = max_over_ranks(rs)
        respaced = {"workload": "config4: timestep_respacing ddim50 (50 of 1000 steps), i2i DDIM (eta 0), one volume "
                                f"per GPU, {'HIP-graph-captured' if args.graph else 'eager'} step",
                    "s_per_volume": round(rs, 4), "denoising_steps_per_s": round(world * 50 / rs, 3)}

    # the production inference path (infer_pod.yml: *_BEST_sampled_10.pt checkpoints,
    # Fast-DDPM 'sampled' schedule with 10 steps), one whole volume, graph loop
    fast10 = None
    if args.respaced:
        from guided_diffusion import script_util
        fd = script_util.create_gaussian_diffusion(steps=10, sample_schedule="sampled", predict_xstart=True, mode="i2i")
        fd.use_hip_graph = bool(args.graph)
        for rep in range(2):   # first pass warms the capture path
            sync()
            t1 = time.perf_counter()
            fd.p_sample_loop(model, tuple(x_T.shape), noise=x_T, cond=cond, progress=False)
            sync()
            rs = time.perf_counter() - t1
        rs = max_over_ranks(rs)
        fast10 = {"workload": "f2: Fast-DDPM production inference (diffusion_steps 10, sample_schedule 'sampled'), "
                              "one volume per GPU, HIP-graph loop",
                  "s_per_volume": round(rs, 4), "denoising_steps_per_s": round(world * 10 / rs, 3)}

    # fp32 parity mode (the numerics the 1e-3 parity tests pin): same weights,
    # same inputs, exact-fp32 MFMA
    fp32 = None
    if args.fp32 and args.dtype != "fp32":
        model.set_compute_dtype("fp32")
        lf = diffusion._native_loop(model, x_T, list(range(T))[::-1][:args.fp32 + 3], cond, True,
                                    graph=bool(args.graph), fresh_outputs=False, need_pred=False)
        tf = max_over_ranks(time_loop(lf, (1, args.fp32), world, sync))
        lf.close()
        model.set_compute_dtype(args.dtype)
        fp32 = {"denoising_steps_per_s": round(world * args.fp32 / tf, 4), "ms_per_step": round(1000 * tf / args.fp32, 2),
                "steps": args.fp32, "mfma_frac_of_fp32_peak": round(step_flops * args.fp32 / tf / 1e12 / F32_PEAK_TFLOPS, 4)}
        torch.cuda.empty_cache()

    # the accurate fast mode: fp32 activations, the wide-grid conv MFMAs on bf16
    # hi/lo splits of both operands (compute_dtype "fp32x"; within the north star's
    # 1e-3 of the reference, tests/test_gpu_fullsize.py)
    split = None
    if args.fp32x and args.dtype != "fp32x":
        model.set_compute_dtype("fp32x")
        lf = diffusion._native_loop(model, x_T, list(range(T))[::-1][:args.fp32x + 3], cond, True,
                                    graph=bool(args.graph), fresh_outputs=False, need_pred=False)
        tf = max_over_ranks(time_loop(lf, (1, args.fp32x), world, sync))
        lf.close()
        model.set_compute_dtype(args.dtype)
        split = {"denoising_steps_per_s": round(world * args.fp32x / tf, 4), "ms_per_step": round(1000 * tf / args.fp32x, 2),
                 "steps": args.fp32x, "mfma_frac_bf16_equiv": round(3 * step_flops * args.fp32x / tf / 1e12 / BF16_PEAK_TFLOPS, 4),
                 "numerics": "fp32 storage; products hi.hi + lo.hi + hi.lo of bf16 splits (3 bf16 MFMA passes per "
                             "16 fp32 channels), fp32 accumulation"}
        torch.cuda.empty_cache()

    # fp16 mode: the same config-2 step with 16-bit IEEE half activations and
    # weights (fp32 accumulation, statistics and diffusion state), the
    # finer-mantissa alternative to bf16 at the same MFMA rate
    fp16 = None
    if args.fp16 and args.dtype != "fp16":
        model.set_compute_dtype("fp16")
        lf = diffusion._native_loop(model, x_T, list(range(T))[::-1][:args.fp16 + 3], cond, True,
                                    graph=bool(args.graph), fresh_outputs=False, need_pred=False)
        tf = max_over_ranks(time_loop(lf, (2, args.fp16), world, sync))
        lf.close()
        model.set_compute_dtype(args.dtype)
        fp16 = {"denoising_steps_per_s": round(world * args.fp16 / tf, 3), "ms_per_step": round(1000 * tf / args.fp16, 3),
                "steps": args.fp16, "mfma_frac": round(step_flops * args.fp16 / tf / 1e12 / BF16_PEAK_TFLOPS, 4)}
        torch.cuda.empty_cache()

    # snapshot for the CPU baseline before the training leg moves the weights
    cpu_state = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu_state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
        cpu_cond, cpu_x = cond.cpu(), x_T.cpu()

    wavunet = None
    if args.wavunet:
        wavunet = wavunet_leg(args, diffusion, x_T, cond, device, world, sync, max_over_ranks)

    config5 = None
    if args.config5:
        config5 = config5_leg(args, device, rank, world, sync, max_over_ranks)

    train5 = None
    if args.train5:
        train5 = train5_leg(args, device, rank, world, sync, max_over_ranks)

    train = None
    if args.train:
        train = train_leg(model, diffusion, n, rank, world, device, args.train, 2, sync, max_over_ranks)

    # HBM bytes of the same conv family per step, from the committed rocprofv3
    # PMC passes of this bench (tools/pmc_traffic.py; FETCH_SIZE x2 on gfx950)
    traffic, traffic_src = None, None
    if n == 128 and args.dtype == "bf16":
        for tj in TRAFFIC_JSONS:
            if os.path.exists(tj):
                with open(tj) as fh:
                    traffic = json.load(fh)["mfma_conv_kernels"]["hbm_bytes"]
                traffic_src = os.path.relpath(tj, ROOT)
                break

    ms_per_step = 1000.0 * elapsed / args.steps
    value = world * args.steps / elapsed
    peak = F32_PEAK_TFLOPS if args.dtype == "fp32" else BF16_PEAK_TFLOPS   # fp16 MFMA: the bf16 rate
    achieved = conv_flops / (conv_ms * 1e-3) / 1e12
    res = {
        "metric": "denoising-steps/sec on 8-ch 128^3 volumes (1000-step DDPM, i2i cWDM)",
        "value": round(value, 4),
        "unit": "denoising-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (seeded 256^3 phantoms -> Haar DWT; seeded non-zero weights)",
        "config": {"workload": "config2: BraTS 3->1 conditional synthesis, 1xMI355X per replica, "
                               f"{n}^3 subbands, 1000-step DDPM (direct linear schedule)",
                   "model": "UNetModel run.sh (mc 64, mult 1,2,2,4,4, 2 res blocks, 81.5M params)",
                   "global_batch": world, "seq_len": n ** 3, "parallelism": f"replicas{world}"},
        "sampling_wallclock_s_per_volume_1000_steps": round(1000 * ms_per_step / 1000.0, 2),
        "hip_graph": bool(args.graph),
        "respaced_ddim50": respaced,
        "fast_ddpm_sampled10": fast10,
        "batched_serving": batched,
        "fp32_parity_mode": fp32,
        "split_bf16_mode": split,
        "fp16_mode": fp16,
        "train_ddp": train,
        "config5_224": config5,
        "train_config5_224": train5,
        "wavunet_128": wavunet,
        "mfma_util_whole_step": round(step_flops * (value / world) / 1e12 / peak, 4),
        "roofline": {"bound": "mfma", "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "traffic_unit": "HBM bytes per step of those launches (2 x FETCH_SIZE + WRITE_SIZE, "
                                     f"{traffic_src})",
                     "kernel": f"implicit-GEMM MFMA conv kernels (conv3d_v5 warp-specialised, conv3d_v4 DMA-staged, conv3d_sg "
                               f"small-grid, brick, head2 output head: "
                               f"{n_conv} launches per step, {conv_ms:.2f} ms, {conv_flops / 1e12:.2f} TFLOP)"},
    }
    if cpu_state is not None:
        threads = cpu_threads()
        dts = cpu_baseline(cpu_state, cpu_cond, cpu_x, threads)
        per = sum(dts) / len(dts)
        res["cpu_baseline"] = {"value": round(1.0 / per, 6), "unit": "denoising-steps/s", "cores": threads,
                               "kind": "port",
                               "sample": f"oracle p_sample (fp32 PyTorch-CPU restatement of the reference path) at "
                                         f"{n}^3 with this run's weights, phantom cond and x_T: 1 warm-up + "
                                         f"{len(dts)} timed steps (t=998, 997), torch threads = the cores this "
                                         f"process may use (affinity/cgroup quota; the host has "
                                         f"{os.cpu_count()} CPUs)",
                               "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
                               "seconds_per_step": [round(d, 2) for d in dts],
                               "extrapolated_s_per_volume": {"1000_steps": round(1000 * per, 1),
                                                             "50_steps": round(50 * per, 1)},
                               "config1_end_to_end_s": round(cpu_config1(threads), 3),
                               "config1_workload": "config 1 on CPU, end to end: 64^3 phantoms -> DWT "
                                                   "conditioning -> 2-step 'sampled' loop, tiny U-Net (mc 32, "
                                                   "mult 1,2) -> IDWT, clamp, mask (oracle.cases.c1_run)"}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
