"""WavUNetModel on the native U-Net plan (drop-in for guided_diffusion/wunet.py:410-795).

The frequency-aware U-Net of the reference (use_freq=True): every ResBlock
that changes resolution does it with a 3D Haar DWT after its first conv (LLL /
3 continues, the 7 high bands become the skip) or an IDWT(3 h, skip bands)
(wunet.py:40-128, :210-269); each encoder level adds a WaveletDownsample of
the input pyramid (:131-145); the decoder has no concatenation.  The reference
builds the decoder with list reuse (:648-687) so one ResBlock per level is
registered twice and runs twice; this class reproduces that state_dict (both
names point at one Parameter) and the plan runs the block twice.

Native path: the same plan as UNetModel (``cwdm_unet_*`` with
``use_freq=1``); the DWT/IDWT resampling, emb add and the GroupNorm
statistics of their outputs run in one channels-last kernel
(``cwdm_haar_nd``), convs on the MFMA kernels.  Training: the plan's backward
(``cwdm_unet_backward``) runs the adjoints -- the DWT's adjoint is the IDWT
and vice versa (orthonormal Haar), the reused decoder blocks' gradients sum
into the owner's parameters -- so ``model(x, t)`` under autograd and
TrainLoop work as for UNetModel.
"""
import torch as th

from .unet import UNetModel


class WavUNetModel(UNetModel):
    use_freq = True

    def __init__(self, image_size, in_channels, model_channels, out_channels, num_res_blocks, attention_resolutions,
                 dropout=0, channel_mult=(1, 2, 4, 8), conv_resample=True, dims=2, num_classes=None,
                 use_checkpoint=False, use_fp16=False, num_heads=1, num_head_channels=-1, num_heads_upsample=-1,
                 use_scale_shift_norm=False, resblock_updown=False, use_new_attention_order=False, num_groups=32,
                 bottleneck_attention=True, resample_2d=True, additive_skips=False, decoder_device_thresh=0,
                 use_freq=False, progressive_input='residual', compute_dtype=None):
        th.nn.Module.__init__(self)
        unsupported = []
        if not use_freq:
            unsupported.append("use_freq=False (the reference's WavUNetModel then skips its high bands; "
                               "use UNetModel)")
        if dims != 3:
            unsupported.append(f"dims={dims} (3D only)")
        if attention_resolutions:
            unsupported.append("attention blocks")
        if bottleneck_attention:
            unsupported.append("bottleneck_attention=True")
        if not resblock_updown:
            unsupported.append("resblock_updown=False (wunet.Downsample with use_freq ignores its conv)")
        if use_scale_shift_norm:
            unsupported.append("use_scale_shift_norm=True")
        if additive_skips:
            unsupported.append("additive_skips=True")
        if progressive_input != 'residual':
            unsupported.append(f"progressive_input={progressive_input!r}")
        if num_classes is not None:
            unsupported.append("class conditioning")
        if dropout:
            unsupported.append("dropout > 0")
        if unsupported:
            raise NotImplementedError("fast-cwdm_amd WavUNetModel covers script_util's use_freq=True "
                                      "configuration; unsupported: " + ", ".join(unsupported))
        # resample_2d has no effect with use_freq (the DWT / IDWT are 3D, wunet.py:76, :120)
        self.progressive_input = progressive_input
        self._setup_native(image_size, in_channels, model_channels, out_channels, num_res_blocks,
                           attention_resolutions, dropout, channel_mult, conv_resample, num_classes, use_checkpoint,
                           num_heads, num_groups, resblock_updown, bottleneck_attention, additive_skips,
                           decoder_device_thresh, compute_dtype)
