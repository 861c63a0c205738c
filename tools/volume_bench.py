"""Front end timing: prepare_modality on a BraTS-size
(240, 240, 155) float64 volume on the GPU vs the reference's numpy
clip_and_normalize + pad + crop on the host (oracle/volume.py)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "fast-cwdm_amd"), ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from guided_diffusion import bratsloader  # noqa: E402
from oracle import volume as ov  # noqa: E402
from test_volume_cpu import brain_like  # noqa: E402


def main():
    img = brain_like((240, 240, 155), 0)
    x = torch.from_numpy(img).cuda()
    for _ in range(3):
        bratsloader.prepare_modality(x)
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        bratsloader.prepare_modality(x)
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    ov.modality_tensor(img)
    cpu = time.perf_counter() - t0
    # algorithmic bytes: 6 radix passes over 71.4 MB + prepare (read 71.4 MB, write 32.1 MB)
    nb = img.nbytes
    algo = 6 * nb + nb + 224 * 224 * 160 * 4
    print(json.dumps({"workload": "prepare_modality (240,240,155) float64 -> (1,224,224,160) fp32",
                      "gpu_ms": round(gpu * 1e3, 3), "cpu_numpy_ms": round(cpu * 1e3, 1),
                      "algorithmic_GBps": round(algo / gpu / 1e9, 1)}))


if __name__ == "__main__":
    main()
