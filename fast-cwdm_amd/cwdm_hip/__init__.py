"""cwdm_hip -- the MI355X-native runtime under the fast-cwdm API mirror.

``_lib`` binds libcwdm.so (include/cwdm.h); ``ops`` wraps the wavelet,
sampler and layout kernels for torch tensors; ``unet_runtime`` drives the
native U-Net plan.
"""
from ._lib import CWDM_BF16, CWDM_F32, CwdmError, LIB_PATH, lib  # noqa: F401
