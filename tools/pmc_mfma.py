"""Effective clock and MFMA-busy fraction per conv launch of one denoising step
from a rocprofv3 PMC pass (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, ...).

clock = GRBM_GUI_ACTIVE / 8 XCDs / wall (MI355X_MICROARCH.md 'DVFS give-back');
mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8) / (256 CUs x 4 SIMDs)
(fraction of SIMD-cycles with the matrix core busy).  usage: pmc_mfma.py DIR [OUT]"""
import collections
import csv
import glob
import sys


def main():
    rows = []
    for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    d = collections.defaultdict(dict)
    meta = {}
    for r in rows:
        k = int(r["Dispatch_Id"])
        d[k][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    ks = sorted(d)
    # the last complete bf16 step: time-embedding launch to the next (the
    # sampler epilogue may live in the output head; an fp16 side leg may follow)
    idx = [k for k in ks if "time_embed_kernel" in meta[k][0]]
    pairs = [(a, b) for a, b in zip(idx[:-1], idx[1:])
             if any("conv3d_v4_kernel<unsigned short" in meta[k][0] for k in ks if a <= k < b)]
    a, b = pairs[-2] if len(pairs) > 1 else pairs[-1]   # not the last: side-leg setup may follow it
    a -= 1   # (the window below is a < k <= b: shift it to a <= k < b)
    b -= 1
    print(f"{'us':>8} {'GHz':>5} {'mfma_busy':>9}  kernel")
    tot_w = tot_busy = tot_cyc = 0.0
    for k in ks:
        if not a < k <= b:
            continue
        name, s, e = meta[k]
        c = d[k]
        dur = e - s
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / cyc / 1024 if cyc else 0.0
        short = name.split("(")[0].split("::")[-1][:48]
        if dur > 20000:
            print(f"{dur / 1e3:8.1f} {cyc / dur:5.2f} {busy:9.3f}  {short}")
        tot_w += dur
        tot_busy += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        tot_cyc += cyc
    print(f"step: {tot_w / 1e3:.1f} us of kernels, mean clock {tot_cyc / tot_w:.2f} GHz, "
          f"MFMA busy {tot_busy / tot_cyc / 1024:.3f} of SIMD-cycles")


if __name__ == "__main__":
    main()
