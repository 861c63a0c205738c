"""Autograd functions for the 3D Haar DWT/IDWT on libcwdm kernels.

Drop-in for DWT_IDWT/DWT_IDWT_Functions.py:115-208 of the reference.  The
reference contracts dense banded matrices with torch.matmul; here each 2x2x2
block is transformed in registers by one HIP thread (cwdm_haar_dwt3d /
cwdm_haar_idwt3d).  Haar is orthonormal, so the backward of the DWT is the IDWT
of the band gradients and vice versa (reference :138-156, :183-208).  The
matrix arguments of the reference signature are accepted and ignored: the
filter is fixed to pywt's Haar taps.
"""
import torch
from torch.autograd import Function

from cwdm_hip import ops


def _dwt(x):
    bands = ops.dwt3d(x)                     # (8, B, C, d, h, w)
    return tuple(bands[k] for k in range(8))


def _idwt(bands):
    return ops.idwt3d_planes(list(bands))


class DWTFunction_3D(Function):
    @staticmethod
    def forward(ctx, input, *matrices):
        ctx.n_extra = len(matrices)
        return _dwt(input)

    @staticmethod
    def backward(ctx, *grads):
        grads = [g if g is not None else None for g in grads]
        ref = next(g for g in grads if g is not None)
        grads = [g if g is not None else torch.zeros_like(ref) for g in grads]
        return (_idwt(grads),) + (None,) * ctx.n_extra


class IDWTFunction_3D(Function):
    @staticmethod
    def forward(ctx, *args):
        bands, matrices = args[:8], args[8:]
        ctx.n_extra = len(matrices)
        return _idwt(bands)

    @staticmethod
    def backward(ctx, grad_output):
        return _dwt(grad_output.contiguous()) + (None,) * ctx.n_extra
