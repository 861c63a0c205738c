"""C-ABI library: loads without a GPU, exports every declared symbol, and its
U-Net plan agrees with the oracle on names/shapes/FLOPs (no compute calls)."""
import ctypes
import math
import os
import re

import pytest
import torch

from conftest import ROOT
from oracle import unet as ou


def _header_functions():
    text = open(os.path.join(ROOT, "include", "cwdm.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(cwdm_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_every_header_symbol():
    from cwdm_hip import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = _header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(_lib.EXPORTED), set(names) ^ set(_lib.EXPORTED)


def test_version_and_error_channel():
    from cwdm_hip import _lib
    L = _lib.lib()
    assert L.cwdm_version() >= 1000
    rc = L.cwdm_unet_param_info(None, 0, None, 0, None, None)
    assert rc == _lib.E_INVALID
    assert b"bad index" in L.cwdm_last_error()


CFGS = [
    dict(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2, channel_mult=(1, 2, 2, 4, 4)),
    dict(in_channels=32, model_channels=32, out_channels=8, num_res_blocks=1, channel_mult=(1, 2)),
    dict(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=1, channel_mult=(1, 2, 4)),
]


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
def test_plan_param_contract_matches_oracle(cfg, dtype):
    from cwdm_hip.unet_runtime import UNetPlan
    plan = UNetPlan(cfg["in_channels"], cfg["model_channels"], cfg["out_channels"], cfg["num_res_blocks"],
                    cfg["channel_mult"], 32 if cfg["model_channels"] >= 64 else 8, dtype)
    want = ou.param_shapes(**cfg)
    got = plan.param_specs
    assert [n for n, _ in got] == [n for n, _ in want]
    assert [tuple(s) for _, s in got] == [tuple(s) for _, s in want]
    assert plan.packed_bytes > 0


def test_production_param_count_and_flops():
    from cwdm_hip.unet_runtime import UNetPlan
    plan = UNetPlan(32, 64, 8, 2, (1, 2, 2, 4, 4), 32, "bf16")
    n = sum(math.prod(s) for _, s in plan.param_specs)
    assert n == 81_511_048
    f = plan.flops(1, 128, 128, 128)
    assert abs(f / 1e12 - 14.98) < 0.01
    assert abs(plan.flops(1, 112, 112, 80) / 1e12 - 7.17) < 0.01
    ws = plan.workspace_bytes(1, 128, 128, 128)
    assert 1e9 < ws < 40e9


def test_grid_divisibility_check():
    from cwdm_hip.unet_runtime import UNetPlan
    plan = UNetPlan(32, 64, 8, 2, (1, 2, 2, 4, 4), 32, "fp32")
    with pytest.raises(AssertionError):
        plan.check_grid(24, 32, 32)


def test_conv_pack_sizes():
    from cwdm_hip import _lib
    L = _lib.lib()
    assert L.cwdm_conv3d_packed_bytes(64, 64, 3, _lib.CWDM_BF16) == 27 * 64 * 64 * 2
    assert L.cwdm_conv3d_packed_bytes(8, 64, 3, _lib.CWDM_F32) == 27 * 32 * 64 * 4   # cout padded to 32
    assert L.cwdm_conv3d_packed_bytes(64, 24, 3, _lib.CWDM_BF16) == -1              # 24 % 16 != 0
    # fp16: the bf16 layout (16-channel K chunks, 2 bytes per element)
    for co, ci, k in ((64, 64, 3), (8, 64, 3), (256, 512, 1)):
        assert L.cwdm_conv3d_packed_bytes(co, ci, k, _lib.CWDM_F16) == L.cwdm_conv3d_packed_bytes(co, ci, k,
                                                                                               _lib.CWDM_BF16)
    assert L.cwdm_conv3d_packed_bytes(64, 64, 3, 7) == -1                            # unknown dtype


def test_fp16_plan_matches_bf16_layout():
    """compute_dtype="fp16": the same topology, packed-weight size and
    workspace as bf16 (both 16-bit), and the torch dtype is float16."""
    from cwdm_hip.unet_runtime import UNetPlan
    a = UNetPlan(32, 64, 8, 2, (1, 2, 2, 4, 4), 32, "bf16")
    b = UNetPlan(32, 64, 8, 2, (1, 2, 2, 4, 4), 32, "fp16")
    assert a.param_specs == b.param_specs
    assert a.packed_bytes == b.packed_bytes
    assert a.workspace_bytes(1, 64, 64, 64) == b.workspace_bytes(1, 64, 64, 64)
    assert b.torch_dtype == torch.float16
    with pytest.raises(ValueError):
        UNetPlan(32, 64, 8, 2, (1, 2, 2, 4, 4), 32, "fp8")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_plan_param_contract_resblock_updown_false(dtype):
    """resblock_updown=False (Downsample stride-2 conv / Upsample nearest+conv,
    reference unet.py:40-100): names and shapes of the plan == the oracle's."""
    from cwdm_hip.unet_runtime import UNetPlan
    cfg = dict(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2, channel_mult=(1, 2, 2, 4, 4))
    plan = UNetPlan(32, 64, 8, 2, (1, 2, 2, 4, 4), 32, dtype, resblock_updown=False)
    want = ou.param_shapes(resblock_updown=False, **cfg)
    assert [(n, tuple(s)) for n, s in plan.param_specs] == [(n, tuple(s)) for n, s in want]
    names = [n for n, _ in want]
    assert "input_blocks.3.0.op.weight" in names and "output_blocks.2.1.conv.weight" in names
    # algorithmic FLOPs: the stride-2 convs count their 27 C taps, not the expanded kernel
    f_true = plan.flops(1, 32, 32, 32)
    import torch.nn.functional as F  # noqa: F401
    down = sum(2 * (32 >> (k + 1)) ** 3 * c * 27 * c for k, c in enumerate((64, 128, 128, 256)))
    up_ref = UNetPlan(32, 64, 8, 2, (1, 2, 2, 4, 4), 32, dtype).flops(1, 32, 32, 32)
    assert f_true < up_ref and f_true > 0 and down > 0


def test_unet_model_accepts_resblock_updown_false():
    from guided_diffusion.unet import UNetModel
    m = UNetModel(image_size=64, in_channels=32, model_channels=32, out_channels=8, num_res_blocks=1,
                  attention_resolutions=(), channel_mult=(1, 2), dims=3, resblock_updown=False,
                  bottleneck_attention=False, resample_2d=False, num_groups=8)
    sd = m.state_dict()
    assert sd["input_blocks.2.0.op.weight"].shape == (32, 32, 3, 3, 3)
    assert sd["output_blocks.1.1.conv.weight"].shape == (64, 64, 3, 3, 3)
    with pytest.raises(NotImplementedError):
        UNetModel(image_size=64, in_channels=32, model_channels=32, out_channels=8, num_res_blocks=1,
                  attention_resolutions=(), channel_mult=(1, 2), dims=3, resblock_updown=False, conv_resample=False,
                  bottleneck_attention=False, resample_2d=False, num_groups=8)


@pytest.mark.parametrize("cfg", [dict(in_channels=32, model_channels=32, out_channels=8, num_res_blocks=2,
                                      channel_mult=(1, 2)),
                                 dict(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2,
                                      channel_mult=(1, 2, 2, 4, 4))])
def test_wavunet_state_dict_matches_oracle(cfg):
    """script_util.create_model(use_freq=True) -> WavUNetModel: the state_dict
    (names, shapes, order) equals the reference's, including the second prefix
    of each reused decoder ResBlock (wunet.py:648-687), and both names share one
    Parameter (parameters() lists it once)."""
    from guided_diffusion import script_util
    from oracle import wunet as ow
    m = script_util.create_model(image_size=128, num_channels=cfg["model_channels"],
                                 num_res_blocks=cfg["num_res_blocks"],
                                 channel_mult=",".join(str(v) for v in cfg["channel_mult"]), attention_resolutions="",
                                 dims=3, num_groups=8, in_channels=32, out_channels=8, bottleneck_attention=False,
                                 resblock_updown=True, use_freq=True)
    sd = m.state_dict(keep_vars=True)
    want = ow.param_shapes(with_aliases=True, **cfg)
    assert [(n, tuple(v.shape)) for n, v in sd.items()] == [(n, tuple(s)) for n, s in want]
    assert len(list(m.parameters())) == len(ow.param_shapes(**cfg))
    for alias, owner in ow.aliases(**cfg).items():
        assert sd[alias + ".in_layers.2.weight"] is sd[owner + ".in_layers.2.weight"]
    if cfg["model_channels"] == 64:
        assert sum(p.numel() for p in m.parameters()) == 90079304
    with pytest.raises(RuntimeError, match="ROCm device"):   # no CPU fallback, with or without autograd
        m(torch.zeros(1, 32, 32, 32, 32), torch.zeros(1))


def test_wavunet_plan_refusals():
    from cwdm_hip.unet_runtime import UNetPlan
    from cwdm_hip._lib import CwdmError
    with pytest.raises(CwdmError, match="resblock_updown"):
        UNetPlan(32, 32, 8, 2, (1, 2), 8, "fp32", resblock_updown=False, use_freq=True)
    with pytest.raises(CwdmError, match="num_res_blocks=1"):
        UNetPlan(32, 32, 8, 1, (1, 2), 8, "fp32", use_freq=True)
    UNetPlan(32, 32, 8, 1, (1, 1), 8, "fp32", use_freq=True)   # equal channels: the reuse is well-formed
    plan = UNetPlan(32, 32, 8, 2, (1, 2), 8, "fp32", use_freq=True)
    with pytest.raises(AssertionError):
        plan.check_grid(16, 16, 6)    # every level downsamples: edges divisible by 2^levels
    plan.check_grid(16, 16, 4)
    assert plan.grad_workspace_bytes(1, 8, 8, 8) > 0   # the plan trains (DWT/IDWT adjoints in the backward)
    # backward segments tile the parameters (head, each block incl. the pyramid convs, conv_in)
    tot = sum(plan.segment_range(s)[1] for s in range(plan.num_segments))
    assert tot == plan.grad_numel
