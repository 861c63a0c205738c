"""Training-step throughput (BASELINE.json config 3: same model, DDP batch 1 per
GPU, RCCL gradient all-reduce over xGMI).

One step = TrainLoop.run_step on a synthetic 4-modality 2N^3 batch: 4 Haar DWTs
+ q_sample into the 32-channel input, native U-Net forward (activations kept),
MSE over the 8 subbands, native backward in segments (with the bucketed
all-reduce overlapped when WORLD_SIZE > 1), fused AdamW over the flat
parameters.  Prints one JSON line on rank 0 with steps/s (all ranks), the
forward/backward conv TFLOP/s and the fraction of the dense bf16 MFMA peak.

usage: python tools/train_bench.py [--grid 128] [--steps 5] [--dtype bf16]
       python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/train_bench.py
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "fast-cwdm_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench import phantom_gpu, seeded_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=128)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    from guided_diffusion import dist_util, script_util, train_util
    os.environ.setdefault("CWDM_LOGDIR", os.path.join(ROOT, "gpurun_out", "train_bench"))
    dist_util.setup_dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = dist_util.dev()
    margs = script_util.run_sh_model_args(diffusion_steps=1000, sample_schedule="direct")
    keys = script_util.model_and_diffusion_defaults().keys()
    model, diffusion = script_util.create_model_and_diffusion(**{k: margs[k] for k in keys},
                                                              compute_dtype=args.dtype)
    seeded_weights(model, 1)
    model.to(dev)
    n2 = 2 * args.grid
    batch = {k: torch.cat([phantom_gpu(n2, 100 * rank + 10 * i + j, dev) for i in range(args.batch)])
             for j, k in enumerate(("t1n", "t1c", "t2w", "t2f"))}
    loop = train_util.TrainLoop(model=model, diffusion=diffusion, data=[batch], batch_size=args.batch,
                                in_channels=32, image_size=n2, microbatch=-1, lr=1e-5, ema_rate="0.9999",
                                log_interval=10 ** 9, contr="t1n", save_interval=10 ** 9, resume_checkpoint="",
                                resume_step=0, mode="i2i", diffusion_steps=1000)
    for _ in range(args.warmup):
        loop.run_step(batch, {})
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, _, _ = loop.run_step(batch, {})
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t)
    plan = model.plan
    g = args.grid
    ffl = plan.flops(args.batch, g, g, g)
    bfl = plan.backward_flops(args.batch, g, g, g)
    per_step = dt / args.steps
    if rank == 0:
        peak = 2500.0 if args.dtype == "bf16" else 157.3
        print(json.dumps({
            "metric": "training steps/s (TrainLoop.run_step, i2i cWDM, 128^3 subbands)",
            "value": round(world * args.batch * args.steps / dt, 4), "unit": "volumes/s",
            "n_gpus": world, "steps": args.steps, "ms_per_step": round(per_step * 1e3, 2),
            "dtype": args.dtype, "grid": g, "batch_per_gpu": args.batch,
            "conv_tflop_per_step": round((ffl + bfl) / 1e12, 2),
            "conv_tflops_achieved": round((ffl + bfl) / per_step / 1e12, 1),
            "mfma_frac": round((ffl + bfl) / per_step / 1e12 / peak, 4),
            "loss": float(loss), "data": "synthetic phantoms; seeded non-zero weights"}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
