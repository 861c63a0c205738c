"""Per-launch timeline of one denoising step from a rocprofv3 kernel trace of
bench.py (a complete step: from one time-embedding launch to the next).
usage: python tools/trace_step.py gpurun_out/TAG/trace [--agg] [--last] [--back=N]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def short(n):
    n = n.replace("void ", "").replace("cwdm::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:60]


def main():
    rows = load(sys.argv[1])
    # steps start at the time-embedding MLP (the first launch of every U-Net
    # forward; the sampler epilogue may live in the output head)
    marks = [i for i, r in enumerate(rows) if "time_embed_kernel" in r["Kernel_Name"]]
    # the last step of the timed (graph-replayed) loop: bench.py ends with one
    # eager profiling step whose setup copies would otherwise land in it
    if "--last" in sys.argv:
        step = rows[marks[-1]:]
    else:
        # the second-to-last complete step of the bf16 headline loop (a side leg,
        # e.g. the fp16 model, may follow it)
        steps = [(a, b) for a, b in zip(marks[:-1], marks[1:])
                 if any("conv3d_v4_kernel<unsigned short" in r["Kernel_Name"] for r in rows[a:b])]
        back = 2
        for arg in sys.argv:
            if arg.startswith("--back="):
                back = int(arg.split("=")[1])   # which step from the end (2: the one before the last)
        a, b = steps[-back] if len(steps) >= back else steps[-1]
        step = rows[a:b]
    tot = 0.0
    agg = defaultdict(lambda: [0, 0.0])
    for i, r in enumerate(step):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        tot += d
        agg[short(r["Kernel_Name"])][0] += 1
        agg[short(r["Kernel_Name"])][1] += d
        if "--agg" not in sys.argv:
            print(f"{d:9.1f} {i:4d} {short(r['Kernel_Name'])} grid={r.get('Grid_Size', '')}")
    print(f"total {tot:.1f} us over {len(step)} launches; wall {(int(step[-1]['End_Timestamp']) - int(step[0]['Start_Timestamp'])) / 1000:.1f} us")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{t:9.1f} us {n:4d}x  {k}")


if __name__ == "__main__":
    main()
