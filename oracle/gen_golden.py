"""Write tests/golden/c1_sampling.npz: the oracle's outputs on config 1
(TEST INFRASTRUCTURE).  Inputs are regenerated from seeds (oracle/cases.py) by
the tests; only outputs and input checksums are stored.

Run:  python -m oracle.gen_golden
"""
import os

import numpy as np
import torch

from . import cases


def main():
    vols, cond, x_T, noises, params = cases.c1_inputs()
    sample, img = cases.c1_run()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "c1_sampling.npz")
    np.savez_compressed(
        out,
        sample=sample.numpy().astype(np.float32),
        image=img.numpy().astype(np.float32),
        cond_sum=np.float64(cond.double().sum()),
        xT_sum=np.float64(x_T.double().sum()),
        param_sum=np.float64(sum(float(p.double().sum()) for p in params.values())),
    )
    print("wrote", out, "sample |.|max", float(sample.abs().max()))


if __name__ == "__main__":
    torch.set_num_threads(8)
    main()
