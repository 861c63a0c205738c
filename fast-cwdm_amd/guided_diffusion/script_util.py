"""Factories and flag plumbing (drop-in for guided_diffusion/script_util.py:1-604).

Same defaults dicts, kwarg names and argparse helpers, so the reference's
scripts and run.sh flag bundles work unchanged.  ``create_model`` builds the
native ``UNetModel``, or with ``use_freq=True`` the native (forward-only)
``WavUNetModel``; the classifier / super-resolution factories are outside the
hot path and raise.
"""
import argparse

from . import gaussian_diffusion as gd
from .respace import SpacedDiffusion, space_timesteps
from .unet import UNetModel

NUM_CLASSES = 2


def diffusion_defaults():
    return dict(
        learn_sigma=False,
        diffusion_steps=1000,
        noise_schedule="linear",
        timestep_respacing="",
        use_kl=False,
        predict_xstart=False,
        rescale_timesteps=False,
        rescale_learned_sigmas=False,
        dataset="brats",
        dims=2,
        num_groups=32,
        in_channels=1,
    )


def model_and_diffusion_defaults():
    res = dict(
        image_size=64,
        num_channels=128,
        num_res_blocks=2,
        num_heads=4,
        num_heads_upsample=-1,
        num_head_channels=-1,
        attention_resolutions="16,8",
        channel_mult="",
        dropout=0.0,
        class_cond=False,
        use_checkpoint=False,
        use_scale_shift_norm=True,
        resblock_updown=True,
        use_fp16=False,
        use_new_attention_order=False,
        dims=2,
        num_groups=32,
        in_channels=1,
        out_channels=0,
        bottleneck_attention=True,
        resample_2d=True,
        additive_skips=False,
        mode="default",
        use_freq=False,
        predict_xstart=False,
        sample_schedule="direct",
    )
    res.update(diffusion_defaults())
    return res


def run_sh_model_args(**overrides):
    """The canonical run.sh COMMON flag bundle (run.sh:109-135) as kwargs for
    create_model_and_diffusion (channels 64, mult 1,2,2,4,4, 3D, i2i, x0-prediction)."""
    args = model_and_diffusion_defaults()
    args.update(dict(
        num_channels=64, class_cond=False, num_res_blocks=2, num_heads=1, learn_sigma=False,
        use_scale_shift_norm=False, attention_resolutions="", channel_mult="1,2,2,4,4", diffusion_steps=1000,
        sample_schedule="direct", noise_schedule="linear", rescale_learned_sigmas=False, rescale_timesteps=False,
        dims=3, num_groups=32, in_channels=32, out_channels=8, bottleneck_attention=False, resample_2d=False,
        additive_skips=False, use_freq=False, predict_xstart=True, image_size=224, mode="i2i"))
    args.update(overrides)
    return args


def create_model_and_diffusion(image_size, class_cond, learn_sigma, num_channels, num_res_blocks, channel_mult,
                               num_heads, num_head_channels, num_heads_upsample, attention_resolutions, dropout,
                               diffusion_steps, noise_schedule, timestep_respacing, use_kl, predict_xstart,
                               rescale_timesteps, rescale_learned_sigmas, use_checkpoint, use_scale_shift_norm,
                               resblock_updown, use_fp16, use_new_attention_order, dims, num_groups, in_channels,
                               out_channels, bottleneck_attention, resample_2d, additive_skips, mode, use_freq,
                               dataset, sample_schedule="direct", compute_dtype=None):
    model = create_model(image_size, num_channels, num_res_blocks, channel_mult=channel_mult, learn_sigma=learn_sigma,
                         class_cond=class_cond, use_checkpoint=use_checkpoint,
                         attention_resolutions=attention_resolutions, num_heads=num_heads,
                         num_head_channels=num_head_channels, num_heads_upsample=num_heads_upsample,
                         use_scale_shift_norm=use_scale_shift_norm, dropout=dropout, resblock_updown=resblock_updown,
                         use_fp16=use_fp16, use_new_attention_order=use_new_attention_order, dims=dims,
                         num_groups=num_groups, in_channels=in_channels, out_channels=out_channels,
                         bottleneck_attention=bottleneck_attention, resample_2d=resample_2d,
                         additive_skips=additive_skips, use_freq=use_freq, compute_dtype=compute_dtype)
    diffusion = create_gaussian_diffusion(steps=diffusion_steps, learn_sigma=learn_sigma, noise_schedule=noise_schedule,
                                          use_kl=use_kl, predict_xstart=predict_xstart,
                                          rescale_timesteps=rescale_timesteps,
                                          rescale_learned_sigmas=rescale_learned_sigmas,
                                          timestep_respacing=timestep_respacing, mode=mode,
                                          sample_schedule=sample_schedule)
    return model, diffusion


def create_model(image_size, num_channels, num_res_blocks, channel_mult="", learn_sigma=False, class_cond=False,
                 use_checkpoint=False, attention_resolutions="16", num_heads=1, num_head_channels=-1,
                 num_heads_upsample=-1, use_scale_shift_norm=False, dropout=0, resblock_updown=True, use_fp16=False,
                 use_new_attention_order=False, num_groups=32, dims=2, in_channels=1, out_channels=0,
                 bottleneck_attention=True, resample_2d=True, additive_skips=False, use_freq=False,
                 compute_dtype=None):
    if not channel_mult:
        if image_size == 512:
            channel_mult = (1, 1, 2, 2, 4, 4)
        elif image_size == 256:
            channel_mult = (1, 2, 2, 4, 4, 4)
        elif image_size == 128:
            channel_mult = (1, 2, 2, 4, 4)
        elif image_size == 64:
            channel_mult = (1, 2, 3, 4)
        else:
            raise ValueError(f"[MODEL] Unsupported image size: {image_size}")
    else:
        if isinstance(channel_mult, str):
            from ast import literal_eval
            channel_mult = literal_eval(channel_mult)
            if isinstance(channel_mult, int):
                channel_mult = (channel_mult,)
        elif isinstance(channel_mult, tuple):
            pass
        else:
            raise ValueError(f"[MODEL] Value for {channel_mult=} not supported")
    attention_ds = []
    if attention_resolutions:
        for res in attention_resolutions.split(","):
            attention_ds.append(image_size // int(res))
    if out_channels == 0:
        out_channels = 2 * in_channels if learn_sigma else in_channels
    if use_freq:
        from .wunet import WavUNetModel
        return WavUNetModel(
            image_size=image_size, in_channels=in_channels, model_channels=num_channels,
            out_channels=out_channels * (1 if not learn_sigma else 2), num_res_blocks=num_res_blocks,
            attention_resolutions=tuple(attention_ds), dropout=dropout, channel_mult=channel_mult,
            num_classes=(NUM_CLASSES if class_cond else None), use_checkpoint=use_checkpoint, use_fp16=use_fp16,
            num_heads=num_heads, num_head_channels=num_head_channels, num_heads_upsample=num_heads_upsample,
            use_scale_shift_norm=use_scale_shift_norm, resblock_updown=resblock_updown,
            use_new_attention_order=use_new_attention_order, dims=dims, num_groups=num_groups,
            bottleneck_attention=bottleneck_attention, additive_skips=additive_skips, use_freq=use_freq,
            compute_dtype=compute_dtype)
    return UNetModel(
        image_size=image_size, in_channels=in_channels, model_channels=num_channels,
        out_channels=out_channels * (1 if not learn_sigma else 2), num_res_blocks=num_res_blocks,
        attention_resolutions=tuple(attention_ds), dropout=dropout, channel_mult=channel_mult,
        num_classes=(NUM_CLASSES if class_cond else None), use_checkpoint=use_checkpoint, use_fp16=use_fp16,
        num_heads=num_heads, num_head_channels=num_head_channels, num_heads_upsample=num_heads_upsample,
        use_scale_shift_norm=use_scale_shift_norm, resblock_updown=resblock_updown,
        use_new_attention_order=use_new_attention_order, dims=dims, num_groups=num_groups,
        bottleneck_attention=bottleneck_attention, additive_skips=additive_skips, resample_2d=resample_2d,
        compute_dtype=compute_dtype)


def create_gaussian_diffusion(*, steps=1000, learn_sigma=False, sigma_small=False, noise_schedule="linear",
                              use_kl=False, predict_xstart=False, rescale_timesteps=False,
                              rescale_learned_sigmas=False, timestep_respacing="", mode="default",
                              sample_schedule="direct", **kwargs):
    kwargs.pop("use_fast_ddpm", None)
    kwargs.pop("fast_ddpm_strategy", None)
    betas = gd.get_named_beta_schedule(noise_schedule, steps, sample_schedule)
    if use_kl:
        loss_type = gd.LossType.RESCALED_KL
    elif rescale_learned_sigmas:
        loss_type = gd.LossType.RESCALED_MSE
    else:
        loss_type = gd.LossType.MSE
    if not timestep_respacing:
        timestep_respacing = [steps]
    return SpacedDiffusion(
        use_timesteps=space_timesteps(steps, timestep_respacing),
        betas=betas,
        model_mean_type=(gd.ModelMeanType.EPSILON if not predict_xstart else gd.ModelMeanType.START_X),
        model_var_type=((gd.ModelVarType.FIXED_LARGE if not sigma_small else gd.ModelVarType.FIXED_SMALL)
                        if not learn_sigma else gd.ModelVarType.LEARNED_RANGE),
        loss_type=loss_type,
        rescale_timesteps=rescale_timesteps,
        mode=mode,
        **kwargs,
    )


def add_dict_to_argparser(parser, default_dict):
    for k, v in default_dict.items():
        v_type = type(v)
        if v is None:
            v_type = str
        elif isinstance(v, bool):
            v_type = str2bool
        parser.add_argument(f"--{k}", default=v, type=v_type)


def args_to_dict(args, keys):
    return {k: getattr(args, k) for k in keys}


def str2bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true", "t", "y", "1"):
        return True
    if v.lower() in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError("boolean value expected")
