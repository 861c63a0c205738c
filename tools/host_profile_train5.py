"""Host-side profile of the config-5 training step: cProfile over K TrainLoop.run_step
calls (the bench's train5 setup), top functions by own time -- where the Python
spends the time the GPU waits on.  usage: python tools/host_profile_train5.py [K]"""
import cProfile
import os
import pstats
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "fast-cwdm_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    args = types.SimpleNamespace(config5_dtype="fp16", train5=K)
    dev = torch.device("cuda", 0)
    holder = {}
    orig = bench.train5_leg

    # run the bench leg's setup + warm-up, then profile K steps of the same loop
    import guided_diffusion.train_util as tu
    real_init = tu.TrainLoop.__init__

    def init(self, *a, **k):
        real_init(self, *a, **k)
        holder["loop"] = self
    tu.TrainLoop.__init__ = init
    orig(args, dev, 0, 1, torch.cuda.synchronize, lambda x: x)
    loop = holder["loop"]
    batch = loop.datal[0]
    prof = cProfile.Profile()
    torch.cuda.synchronize()
    prof.enable()
    for _ in range(K):
        loop.run_step(batch, {})
    torch.cuda.synchronize()
    prof.disable()
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
