"""fast-cwdm_amd's guided_diffusion: the reference's Python API surface
(script_util / gaussian_diffusion / respace / unet / train_util / dist_util)
over MI355X-native kernels (libcwdm.so through cwdm_hip)."""
