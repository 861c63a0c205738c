"""BraTS volume front end on the device (reference: guided_diffusion/bratsloader.py).

The reference decodes each NIfTI modality in DataLoader worker processes and
runs clip_and_normalize in numpy (bratsloader.py:116-120: two np.quantile
sorts of 8.9 M float64 voxels per modality, then clip and min-max), pads z
155 -> 160 and crops x/y by 8 (:44-50).  Here the decoded array goes to the
GPU once and the rest is libcwdm kernels (cwdm_quantiles: exact order
statistics by radix select; cwdm_volume_prepare: clip + normalise + pad +
crop in one pass), so the step before the wavelet path no longer serialises
on host cores.  Results equal the reference's bit for bit (float64
arithmetic, numpy's 'linear' interpolation; tests/test_gpu_volume.py).
"""
import os

import torch

from cwdm_hip import ops

SEQTYPES = ("t1n", "t1c", "t2w", "t2f", "seg")


def clip_and_normalize(img):
    """bratsloader.py:116-120 on a device tensor; returns float64 like numpy."""
    x = torch.as_tensor(img)
    ops._need_cuda(x)
    lohi = ops.quantiles(x, (0.001, 0.999))
    return ops.volume_prepare(x, lohi, crop=0, out_z=x.shape[-1], out_dtype=torch.float64)


def prepare_modality(img, pad_z=160, crop=8):
    """The per-modality tensor of BRATSVolumes.__getitem__ (bratsloader.py:44-50):
    (1, X - 2 crop, Y - 2 crop, pad_z) fp32 = clip_and_normalize(img) cast to
    fp32, zero-padded in z and cropped in x/y, in one kernel after the quantiles."""
    x = torch.as_tensor(img)
    ops._need_cuda(x)
    if x.dim() != 3:
        raise AssertionError("expected one (X, Y, Z) modality volume")
    lohi = ops.quantiles(x, (0.001, 0.999))
    return ops.volume_prepare(x, lohi, crop=crop, out_z=pad_z, out_dtype=torch.float32).unsqueeze(0)


def finish_sample(sample, cond_1=None, keep_z=155):
    """scripts/sample.py:113-135: IDWT of the sampled subbands (LLL x 3), clamp
    to [0, 1], zero outside the brain (cond_1 == 0), crop z to keep_z;
    returns (B, X, Y, keep_z)."""
    return ops.sample_finish(sample, cond_1, keep_z)


def _prepare_modality_host(img, pad_z=160, crop=8):
    """prepare_modality for DataLoader worker processes, which cannot own a HIP
    context: the reference's own numpy arithmetic (bratsloader.py:40-50,
    116-120) on the host.  Data plumbing either side of the hot path, never
    the sampling/training step itself."""
    import numpy as np
    a = np.asarray(img, dtype=np.float64)
    c = np.clip(a, np.quantile(a, 0.001), np.quantile(a, 0.999))
    c = (c - np.min(c)) / (np.max(c) - np.min(c))
    X, Y, Z = a.shape
    out = torch.zeros(1, X, Y, pad_z)
    out[:, :, :, :Z] = torch.tensor(c)
    return out[:, crop:X - crop, crop:Y - crop, :].contiguous()


class BRATSVolumes(torch.utils.data.Dataset):
    """Same directory walk and item dict as the reference (bratsloader.py:9-113);
    decoding needs nibabel (not part of this image).  In the main process the
    normalisation runs on ``device`` through prepare_modality; inside a
    DataLoader worker (the reference scripts use num_workers=12, and a forked
    worker cannot initialise the GPU) it runs the reference's numpy arithmetic
    on the host and returns CPU tensors, which the caller moves with
    ``.to(dev)`` exactly as the reference scripts do."""

    def __init__(self, directory, mode="train", gen_type=None, device="cuda"):
        super().__init__()
        self.mode = mode
        self.directory = os.path.expanduser(directory)
        self.gentype = gen_type
        self.seqtypes = list(SEQTYPES)
        self.seqtypes_set = set(self.seqtypes)
        self.device = device
        self.database = []
        for root, dirs, files in os.walk(self.directory):
            if not dirs:
                files.sort()
                datapoint = {}
                for f in files:
                    seqtype = f.split("-")[4].split(".")[0]
                    datapoint[seqtype] = os.path.join(root, f)
                self.database.append(datapoint)

    def __len__(self):
        return len(self.database)

    def __getitem__(self, x):
        import nibabel  # the reference's NIfTI decoder; absent here -> ImportError
        filedict = self.database[x]
        missing = "none"
        out = {}
        in_worker = torch.utils.data.get_worker_info() is not None
        for key in ("t1n", "t1c", "t2w", "t2f"):
            if key in filedict:
                arr = nibabel.load(filedict[key]).get_fdata()
                if in_worker or not str(self.device).startswith("cuda"):
                    out[key] = _prepare_modality_host(arr)
                else:
                    out[key] = prepare_modality(torch.from_numpy(arr).to(self.device))
            else:
                missing = key
                out[key] = torch.zeros(1)
        if self.mode in ("eval", "auto"):
            subj = filedict["t1n"] if "t1n" in filedict else filedict["t2f"]
        else:
            subj = "dummy_string"
        out.update({"missing": missing, "subj": subj, "filedict": filedict})
        return out
