"""Counters of a rocprofv3 --pmc pass summed per kernel name, with the MFMA-busy
fraction and the shader clock where those counters are present.
usage: python tools/pmc_by_kernel.py DIR [FILTER]"""
import collections
import csv
import glob
import sys


def main():
    rows = []
    for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    wall = collections.defaultdict(float)
    n = collections.Counter()
    seen = set()
    for r in rows:
        k = r["Kernel_Name"].replace("void ", "").replace("cwdm::", "").split("(")[0][:60]
        if flt not in k:
            continue
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        did = r["Dispatch_Id"]
        if did not in seen:
            seen.add(did)
            n[k] += 1
            wall[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for k in sorted(per, key=lambda q: -wall[q]):
        c = per[k]
        s = f"{k:60s} {n[k]:4d}x {wall[k]:9.1f} us"
        if "GRBM_GUI_ACTIVE" in c:
            gui = c["GRBM_GUI_ACTIVE"] / 8
            s += f"  clk {gui / wall[k] / 1e3:.2f} GHz"
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                s += f"  mfma_busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / gui / 1024:.3f}"
        s += "  " + " ".join(f"{q}={v:.4g}" for q, v in sorted(c.items()) if q not in ("GRBM_GUI_ACTIVE",))
        print(s)


if __name__ == "__main__":
    main()
