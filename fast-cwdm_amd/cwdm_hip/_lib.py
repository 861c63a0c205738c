"""ctypes binding of libcwdm.so (include/cwdm.h).

The library is built in-tree (``fast-cwdm_amd/lib/libcwdm.so``) by
``__graft_entry__.build()`` / ``make -C fast-cwdm_amd/csrc``.  There is no
fallback: if the library is missing or a call fails, this module raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CWDM_LIB", os.path.join(_HERE, "..", "lib", "libcwdm.so"))

CWDM_F32 = 0
CWDM_BF16 = 1
CWDM_F64 = 2
CWDM_F16 = 3

E_INVALID, E_SHAPE, E_HIP, E_WORKSPACE, E_INDEX, E_UNSUPPORTED = -1, -2, -3, -4, -5, -6

i64 = ctypes.c_int64
vp = ctypes.c_void_p
I64x3 = i64 * 3
I64x4 = i64 * 4


class SamplerArgs(ctypes.Structure):
    _fields_ = [
        ("model_out", vp), ("mo_s", I64x3),
        ("x_t", vp), ("xt_s", I64x3),
        ("x_prev", vp), ("xp_s", I64x3),
        ("noise", vp), ("nz_s", I64x3),
        ("pred_xstart", vp), ("px_s", I64x3),
        ("mirror", vp), ("mirror_dtype", ctypes.c_int), ("mr_s", I64x3),
        ("coef", vp), ("t", vp),
        ("T", i64), ("B", i64), ("d", i64), ("h", i64), ("w", i64),
        ("clip_denoised", ctypes.c_int),
        ("mean_type", ctypes.c_int),
        ("update", ctypes.c_int),
        ("per_band", ctypes.c_int),
        ("levels", ctypes.c_int),
        ("noise_philox", ctypes.c_int),
        ("reserved0", ctypes.c_int),
        ("noise_seed", ctypes.c_uint64),
    ]


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int),
        ("B", i64), ("D", i64), ("H", i64), ("W", i64),
        ("cout", ctypes.c_int),
        ("a0", vp), ("a_c0", ctypes.c_int),
        ("a1", vp), ("a_c1", ctypes.c_int),
        ("a_mode", ctypes.c_int),
        ("a_gn", vp),
        ("a_w", vp),
        ("b0", vp), ("b_c0", ctypes.c_int),
        ("b1", vp), ("b_c1", ctypes.c_int),
        ("b_w", vp),
        ("bias", vp), ("bias_bstride", i64),
        ("res", vp), ("res_mode", ctypes.c_int),
        ("out", vp), ("out_dtype", ctypes.c_int),
        ("stats", vp),
        ("workspace", vp), ("ws_bytes", i64),
        ("out1", vp), ("out_c0", ctypes.c_int),
        ("accumulate", ctypes.c_int),
        ("a_w_split", vp),
    ]


class WgradDesc(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int),
        ("B", i64), ("D", i64), ("H", i64), ("W", i64),
        ("ksize", ctypes.c_int),
        ("u0", vp), ("u_c0", ctypes.c_int),
        ("u1", vp), ("u_c1", ctypes.c_int),
        ("u_mode", ctypes.c_int),
        ("u_gn", vp),
        ("dy", vp), ("dy_cs", ctypes.c_int), ("cout", ctypes.c_int),
        ("dw", vp),
        ("workspace", vp),
        ("u_cm", ctypes.c_int),
        ("ws_bytes", i64),
    ]


class UNetConfig(ctypes.Structure):
    _fields_ = [
        ("in_channels", ctypes.c_int), ("model_channels", ctypes.c_int),
        ("out_channels", ctypes.c_int), ("num_res_blocks", ctypes.c_int),
        ("num_levels", ctypes.c_int), ("channel_mult", ctypes.c_int * 8),
        ("num_groups", ctypes.c_int), ("dtype", ctypes.c_int),
        ("resblock_updown", ctypes.c_int), ("use_freq", ctypes.c_int),
        ("mfma_split", ctypes.c_int),
    ]


class HaarNdDesc(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int),
        ("B", i64), ("d", i64), ("h", i64), ("w", i64),
        ("C", ctypes.c_int),
        ("inverse", ctypes.c_int),
        ("src", vp), ("high_in", vp),
        ("lll_scale", ctypes.c_float), ("high_scale", ctypes.c_float),
        ("out", vp), ("all8", ctypes.c_int), ("high_out", vp),
        ("bias", vp), ("bias_bstride", i64),
        ("stats", vp),
    ]


# name -> (restype, argtypes)
_PROTOS = {
    "cwdm_version": (ctypes.c_int, []),
    "cwdm_last_error": (ctypes.c_char_p, []),
    "cwdm_build_id": (ctypes.c_char_p, []),
    "cwdm_haar_dwt3d": (ctypes.c_int, [vp, i64, i64, i64, i64, i64, vp, ctypes.c_int, ctypes.POINTER(i64),
                                       ctypes.c_int, vp]),
    "cwdm_haar_idwt3d": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(i64), i64, i64, i64, i64, i64, vp,
                                        ctypes.c_int, ctypes.c_int, vp]),
    "cwdm_haar_idwt3d_planes": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(i64), i64, i64, i64,
                                               i64, i64, vp, vp]),
    "cwdm_prepare_batch": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i64, i64, i64, vp, ctypes.c_int, vp, i64, vp, vp,
                                          vp]),
    "cwdm_prepare_batch2": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i64, i64, i64, vp, ctypes.c_int, vp, i64, vp, vp,
                                           vp]),
    "cwdm_sampler_step": (ctypes.c_int, [ctypes.POINTER(SamplerArgs), vp]),
    "cwdm_quantile_workspace_bytes": (i64, []),
    "cwdm_quantiles": (ctypes.c_int, [vp, ctypes.c_int, i64, ctypes.POINTER(i64), ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double), vp, vp, i64, vp]),
    "cwdm_volume_prepare": (ctypes.c_int, [vp, ctypes.c_int, i64, i64, i64, vp, i64, i64, vp, ctypes.c_int, vp]),
    "cwdm_sample_finish": (ctypes.c_int, [vp, i64, i64, i64, i64, vp, i64, vp, vp]),
    "cwdm_copy3": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(i64), vp, ctypes.c_int, ctypes.POINTER(i64),
                                  i64, i64, i64, vp]),
    "cwdm_conv3d_packed_bytes": (i64, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "cwdm_conv3d_pack": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]),
    "cwdm_conv3d_packed_split_bytes": (i64, [ctypes.c_int, ctypes.c_int]),
    "cwdm_conv3d_pack_split": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, vp, vp]),
    "cwdm_conv3d_pack_dgrad": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]),
    "cwdm_conv3d_parts": (i64, [ctypes.c_int, i64, i64, i64, ctypes.c_int]),
    "cwdm_space_to_depth": (ctypes.c_int, [vp, ctypes.c_int, i64, i64, i64, i64, ctypes.c_int, vp, ctypes.c_int,
                                           ctypes.c_int, vp]),
    "cwdm_conv3d_pack_s2": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp]),
    "cwdm_conv3d_s2_fold_dw": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp]),
    "cwdm_conv3d_forward": (ctypes.c_int, [ctypes.POINTER(ConvDesc), vp]),
    "cwdm_conv3d_workspace_bytes": (i64, [ctypes.POINTER(ConvDesc)]),
    "cwdm_gn_finalize": (ctypes.c_int, [vp, i64, ctypes.c_int, vp, i64, ctypes.c_int, vp, vp, ctypes.c_int, i64, i64,
                                        ctypes.c_float, vp, vp, vp]),
    "cwdm_gn_silu_pool": (ctypes.c_int, [vp, ctypes.c_int, vp, i64, i64, i64, i64, ctypes.c_int, vp, vp, vp]),
    "cwdm_gn_apply": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_int, vp, i64, i64, ctypes.c_int, vp, vp]),
    "cwdm_conv3d_set_path": (ctypes.c_int, [ctypes.c_int]),
    "cwdm_debug_v5_grid": (ctypes.c_int, [ctypes.c_int]),
    "cwdm_debug_v5_aa": (ctypes.c_int, [ctypes.c_int]),
    "cwdm_debug_v5_aa_timeout": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "cwdm_device_status": (ctypes.c_int, [ctypes.c_int]),
    "cwdm_debug_gn_fin_apply": (ctypes.c_int, [vp, i64, ctypes.c_int, vp, i64, ctypes.c_int, vp, vp, ctypes.c_int,
                                               i64, i64, ctypes.c_float, vp, vp, ctypes.c_int, vp, vp, vp, vp]),
    "cwdm_debug_head2": (ctypes.c_int, [ctypes.c_int]),
    "cwdm_debug_pw_lt": (ctypes.c_int, [ctypes.c_int]),
    "cwdm_debug_conv_stamps": (ctypes.c_int, [vp]),
    "cwdm_conv3d_wgrad": (ctypes.c_int, [ctypes.POINTER(WgradDesc), vp]),
    "cwdm_conv3d_wgrad_workspace_bytes": (i64, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "cwdm_gn_silu_bwd_workspace_bytes": (i64, [ctypes.c_int, i64, i64, i64, i64]),
    "cwdm_gn_silu_bwd": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_int, vp, ctypes.c_int, vp, vp, vp,
                                        ctypes.c_int, i64, i64, i64, i64, ctypes.c_int, vp, ctypes.c_int, vp,
                                        ctypes.c_int, vp, vp, vp, i64, vp]),
    "cwdm_resample_add": (ctypes.c_int, [vp, vp, ctypes.c_int, i64, i64, i64, i64, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, vp]),
    "cwdm_channel_sum_workspace_bytes": (i64, [i64, i64, ctypes.c_int]),
    "cwdm_channel_sum": (ctypes.c_int, [vp, ctypes.c_int, i64, i64, ctypes.c_int, ctypes.c_int, vp, i64, vp, vp,
                                        vp, i64, vp]),
    "cwdm_adamw": (ctypes.c_int, [vp, vp, vp, vp, i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_double, ctypes.c_double, i64, vp]),
    "cwdm_adamw_device_step": (ctypes.c_int, [vp, vp, vp, vp, i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                               ctypes.c_double, ctypes.c_double, vp, vp, vp]),
    "cwdm_adamw_maxabs": (ctypes.c_int, [vp, vp, vp, vp, i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_double, i64, vp, vp]),
    "cwdm_unet_create": (ctypes.c_int, [ctypes.POINTER(UNetConfig), ctypes.POINTER(vp)]),
    "cwdm_unet_destroy": (None, [vp]),
    "cwdm_unet_num_params": (ctypes.c_int, [vp]),
    "cwdm_unet_num_aliases": (ctypes.c_int, [vp]),
    "cwdm_unet_alias_info": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "cwdm_haar_nd_parts": (i64, [i64, i64, i64]),
    "cwdm_haar_nd": (ctypes.c_int, [ctypes.POINTER(HaarNdDesc), vp]),
    "cwdm_wavelet2_analysis": (ctypes.c_int, [vp, i64, i64, i64, i64, vp, ctypes.c_int, i64, i64, ctypes.c_int, vp]),
    "cwdm_wavelet2_synthesis": (ctypes.c_int, [vp, i64, i64, i64, i64, i64, i64, ctypes.c_int, vp, vp]),
    "cwdm_unet_param_info": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(i64),
                                            ctypes.POINTER(ctypes.c_int)]),
    "cwdm_unet_packed_bytes": (i64, [vp]),
    "cwdm_unet_pack": (ctypes.c_int, [vp, ctypes.POINTER(vp), vp, vp]),
    "cwdm_unet_workspace_bytes": (i64, [vp, i64, i64, i64, i64]),
    "cwdm_unet_train_workspace_bytes": (i64, [vp, i64, i64, i64, i64]),
    "cwdm_unet_forward": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i64, i64, i64, vp, i64, vp]),
    "cwdm_unet_forward_step": (ctypes.c_int, [vp, vp, vp, vp, ctypes.POINTER(SamplerArgs), i64, i64, i64, i64,
                                              vp, i64, ctypes.POINTER(ctypes.c_int), vp]),
    "cwdm_unet_trace_count": (ctypes.c_int, [vp]),
    "cwdm_unet_trace_info": (ctypes.c_int, [vp, ctypes.c_int, i64, i64, i64, i64, ctypes.POINTER(i64),
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "cwdm_unet_flops": (ctypes.c_double, [vp, i64, i64, i64, i64]),
    "cwdm_unet_packed_bwd_bytes": (i64, [vp]),
    "cwdm_unet_pack_bwd": (ctypes.c_int, [vp, ctypes.POINTER(vp), vp, vp]),
    "cwdm_unet_grad_workspace_bytes": (i64, [vp, i64, i64, i64, i64]),
    "cwdm_unet_backward_segments": (ctypes.c_int, [vp]),
    "cwdm_unet_segment_range": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
    "cwdm_unet_backward": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, vp, i64, vp, i64,
                                          ctypes.c_int, ctypes.c_int, vp]),
    "cwdm_unet_backward_flops": (ctypes.c_double, [vp, i64, i64, i64, i64]),
    "cwdm_unet_set_profiling": (ctypes.c_int, [vp, ctypes.c_int]),
    "cwdm_unet_profile_read": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_int)]),
}

EXPORTED = tuple(_PROTOS)

_lib = None


class CwdmError(RuntimeError):
    pass


def lib():
    """Load libcwdm.so once (raises OSError if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"libcwdm.so not found at {LIB_PATH}: run __graft_entry__.build() "
                          f"or `make -C fast-cwdm_amd/csrc` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        check_build_id(L)
        _lib = L
    return _lib


def check_build_id(L):
    """Refuse a library built from other sources than the tree's (the .so is
    untracked and travels to the GPU box as a file; CWDM_ALLOW_STALE_LIB=1
    skips the check for kernel experiments)."""
    from .srchash import source_files, source_hash
    if os.environ.get("CWDM_ALLOW_STALE_LIB") == "1":
        return
    if not all(os.path.exists(f) for f in source_files_or_empty(source_files)):
        # a deployment that ships only the .so: nothing to compare against
        import warnings
        warnings.warn(f"libcwdm sources not found next to the package: build id of {LIB_PATH} not checked")
        return
    built = L.cwdm_build_id().decode()
    want = source_hash()
    if built != want:
        raise OSError(f"{LIB_PATH} was built from sources {built}, the tree has {want}: "
                      f"rebuild with `make -C fast-cwdm_amd/csrc`")


def source_files_or_empty(source_files):
    """The source list the build id covers, or [""] (a path that does not
    exist) when the csrc directory itself is absent."""
    try:
        return source_files()
    except OSError:
        return [""]


def check(rc, what=""):
    """Map a CWDM_E_* return code to the reference's exception types."""
    if rc == 0:
        return
    msg = lib().cwdm_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == E_SHAPE:
        raise AssertionError(text)
    if rc == E_INDEX:
        raise IndexError(text)
    if rc == E_INVALID:
        raise ValueError(text)
    raise CwdmError(f"{text} (code {rc})")


def strides(*s):
    return (i64 * len(s))(*[int(v) for v in s])
