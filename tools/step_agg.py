"""Per-kernel aggregate of one step in a rocprofv3 kernel trace, the step
delimited by two launches of a marker kernel (the last two by default).
usage: python tools/step_agg.py TRACE.csv MARKER_SUBSTRING [--list] [--nth K]"""
import csv
import sys
from collections import defaultdict


def short(n):
    n = n.replace("cwdm::", "").replace("(anonymous namespace)::", "").replace("unsigned short", "u16")
    return n.split("(")[0][:90]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
mk = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
nth = int(sys.argv[sys.argv.index("--nth") + 1]) if "--nth" in sys.argv else 1
a, b = mk[-1 - nth] + 1, mk[-nth] + 1
step = rows[a:b]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
agg = defaultdict(lambda: [0.0, 0])
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = short(r["Kernel_Name"])
    agg[k][0] += d
    agg[k][1] += 1
busy = sum(v[0] for v in agg.values())
print(f"step: {len(step)} launches, kernel time {busy/1e3:.3f} ms, wall {(t1-t0)/1e6:.3f} ms")
for k, (d, n) in sorted(agg.items(), key=lambda x: -x[1][0]):
    print(f"{d:9.1f} us {n:5d}x  {k}")
if "--list" in sys.argv:
    for i, r in enumerate(step):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"{i:4d} {d:9.1f} {short(r['Kernel_Name'])} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} wg={r['Workgroup_Size_X']}")
