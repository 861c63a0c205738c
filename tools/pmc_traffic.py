"""HBM traffic of the conv family of one denoising step from two rocprofv3 PMC
passes of bench.py (FETCH_SIZE and WRITE_SIZE, each its own run).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3):
FETCH_SIZE (KB) counts half the bytes of 16-B/lane streaming reads on gfx950,
so read bytes = 2 x FETCH_SIZE; WRITE_SIZE (KB) is exact for 16-B stores.

The "dominant kernel" of bench.py's roofline is every launch bracketed by the
plan's per-conv events (conv kernels, their GroupNorm/skip pre-passes, split-K
sums/reduces, the output head, which also runs the fused sampler epilogue).
The step is the last complete bf16 one between two time-embedding launches.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import glob
import json
import sys

CONV_FAMILY = ("conv3d_v5_kernel", "conv3d_v4_kernel", "conv3d_sg_kernel", "conv3d_kernel", "conv3d_wide_kernel",
               "conv3d_reduce_kernel", "splitk_sum_kernel", "gn_apply_kernel", "gn_apply_skip_kernel", "gn_fin_apply_kernel",
               "head_conv_kernel", "head2_kernel")


def last_step(d, counter):
    """The last complete bf16 step: from one time-embedding launch (the first of
    every U-Net forward) to the next, whose convs are the bf16 ones (bench.py
    may run an fp16 side leg after the headline loop)."""
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    idx = [i for i, r in enumerate(rows) if "time_embed_kernel" in r["Kernel_Name"]]
    steps = [rows[a:b] for a, b in zip(idx[:-1], idx[1:])
             if any(("conv3d_v4_kernel<unsigned short" in r["Kernel_Name"] or "conv3d_v5_kernel<unsigned short" in r["Kernel_Name"])
                    for r in rows[a:b])]
    if steps:
        return steps[-2] if len(steps) > 1 else steps[-1]   # not the last: side-leg setup may follow it
    raise SystemExit("no complete bf16 step in " + d)


def short(name):
    for k in CONV_FAMILY:
        if k in name:
            return k
    return None


def main():
    fdir, wdir, out = sys.argv[1:4]
    fr, wr = last_step(fdir, "FETCH_SIZE"), last_step(wdir, "WRITE_SIZE")
    assert [r["Kernel_Name"] for r in fr] == [r["Kernel_Name"] for r in wr], "passes disagree on the launch list"
    per = {}
    tot_r = tot_w = 0.0
    n = 0
    for f, w in zip(fr, wr):
        k = short(f["Kernel_Name"])
        if k is None:
            continue
        rb = 2.0 * float(f["Counter_Value"]) * 1024
        wb = float(w["Counter_Value"]) * 1024
        tot_r += rb
        tot_w += wb
        n += 1
        e = per.setdefault(k, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += rb
        e[2] += wb
    mfma = ("conv3d_v5_kernel", "conv3d_v4_kernel", "conv3d_sg_kernel", "conv3d_kernel", "conv3d_wide_kernel",
            "head_conv_kernel", "head2_kernel")
    mk = {k: v for k, v in per.items() if k in mfma}
    res = {"scope": "conv family of one 128^3 bf16 denoising step (bench.py)", "launches": n,
           "mfma_conv_kernels": {"kernels": sorted(mk), "launches": sum(v[0] for v in mk.values()),
                                 "hbm_bytes": sum(v[1] + v[2] for v in mk.values())},
           "read_bytes": tot_r, "write_bytes": tot_w, "hbm_bytes": tot_r + tot_w,
           "correction": "read = 2 x FETCH_SIZE(KB) x 1024; write = WRITE_SIZE(KB) x 1024 (MI355X_MICROARCH.md)",
           "per_kernel": {k: {"launches": v[0], "read_bytes": v[1], "write_bytes": v[2]} for k, v in per.items()}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("launches", "read_bytes", "write_bytes", "hbm_bytes")}))
    for k, v in per.items():
        print(f"  {k:24s} n={v[0]:3d} read {v[1] / 1e9:8.3f} GB  write {v[2] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
