"""Kernel-by-kernel timeline of the last denoising step in a rocprofv3 .db
(between the last two sampler_kernel launches).  usage: prof_timeline.py <db>"""
import glob, sqlite3, sys, re

path = sys.argv[1]
if not path.endswith(".db"):
    path = glob.glob(path + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(path)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
disp = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
sym = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
cols = [r[1] for r in c.execute(f"pragma table_info({disp})")]
gx = "grid_size_x" if "grid_size_x" in cols else None
q = f"select s.display_name, d.start, d.end{', d.' + gx if gx else ''} from {disp} d join {sym} s on d.kernel_id = s.id order by d.start"
rows = c.execute(q).fetchall()
idx = [i for i, r in enumerate(rows) if "sampler_kernel" in r[0]]
a, b = idx[-2] + 1, idx[-1] + 1
t0 = rows[a][1]
tot = 0
for r in rows[a:b]:
    n = re.sub(r"\(anonymous namespace\)::", "", r[0]).split("(")[0].replace("void ", "").replace("cwdm::", "")
    dt = (r[2] - r[1]) / 1e3
    tot += dt
    print(f"{(r[1]-t0)/1e3:9.1f} {dt:8.1f}us {r[3] if gx else '':>8} {n[:70]}")
print(f"busy {tot/1e3:.3f} ms, wall {(rows[b-1][2]-t0)/1e6:.3f} ms")
