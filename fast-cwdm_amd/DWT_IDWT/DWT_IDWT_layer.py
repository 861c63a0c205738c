"""DWT_3D / IDWT_3D modules (drop-in for DWT_IDWT/DWT_IDWT_layer.py:432-646).

Same constructor (`DWT_3D('haar')`), same forward contracts and asserts:
  DWT_3D()(x[N, C, D, H, W]) -> (LLL, LLH, LHL, LHH, HLL, HLH, HHL, HHH),
  IDWT_3D()(*8 bands) -> x,
with band letters indexing (D, H, W).  Unlike the reference there is no
per-call matrix construction or host->device upload (:505-511): the transform is
one HBM-bound HIP kernel each way.  Only the Haar wavelet -- the one the
fast-cwdm hot path uses -- is implemented.
"""
from torch.nn import Module

from .DWT_IDWT_Functions import DWTFunction_3D, IDWTFunction_3D


def _check_wavelet(name):
    if name != "haar":
        raise NotImplementedError(f"fast-cwdm_amd implements the Haar wavelet only (got {name!r})")


class DWT_3D(Module):
    def __init__(self, wavename):
        super().__init__()
        _check_wavelet(wavename)
        self.wavename = wavename

    def forward(self, input):
        assert len(input.size()) == 5
        self.input_depth, self.input_height, self.input_width = input.shape[-3:]
        return DWTFunction_3D.apply(input)


class IDWT_3D(Module):
    def __init__(self, wavename):
        super().__init__()
        _check_wavelet(wavename)
        self.wavename = wavename

    def forward(self, LLL, LLH, LHL, LHH, HLL, HLH, HHL, HHH):
        assert len(LLL.size()) == len(LLH.size()) == len(LHL.size()) == len(LHH.size()) == 5
        assert len(HLL.size()) == len(HLH.size()) == len(HHL.size()) == len(HHH.size()) == 5
        self.input_depth = LLL.size()[-3] + HHH.size()[-3]
        self.input_height = LLL.size()[-2] + HHH.size()[-2]
        self.input_width = LLL.size()[-1] + HHH.size()[-1]
        return IDWTFunction_3D.apply(LLL, LLH, LHL, LHH, HLL, HLH, HHL, HHH)


class DWT_3D_Multilevel(Module):
    """J-level Haar analysis for the multi-level wavelet diffusion of BASELINE
    config 5 (no reference module: README.md:3-9 names it).
    forward(x) -> [LLL_J, {LLH..HHH} level J, ..., level 1] (pywt.wavedecn
    order and semantics, band letters in (D, H, W) order)."""

    def __init__(self, wavename, level=2):
        super().__init__()
        _check_wavelet(wavename)
        self.wavename, self.level = wavename, level

    def forward(self, input):
        from cwdm_hip import ops
        return ops.wavedec3(input, self.level)


class IDWT_3D_Multilevel(Module):
    """Inverse of DWT_3D_Multilevel (pywt.waverecn)."""

    def __init__(self, wavename):
        super().__init__()
        _check_wavelet(wavename)
        self.wavename = wavename

    def forward(self, coeffs):
        from cwdm_hip import ops
        return ops.waverec3(coeffs)
