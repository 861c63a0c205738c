"""Per-kernel summary of a rocprofv3 results .db (kernel trace): calls, total, avg, max (us).
usage: prof_db.py <run_results.db> [steps]  -- per-step ms when steps given."""
import glob, sqlite3, sys
from collections import defaultdict

path = sys.argv[1]
if not path.endswith(".db"):
    path = glob.glob(path + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(path)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
disp = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
sym = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
cols = [r[1] for r in c.execute(f"pragma table_info({sym})")]
namecol = "display_name" if "display_name" in cols else "kernel_name"
rows = c.execute(f"select s.{namecol}, d.start, d.end from {disp} d join {sym} s on d.kernel_id = s.id").fetchall()
agg = defaultdict(list)
for n, s, e in rows:
    agg[n.split("(")[0][:90]].append((e - s) / 1e3)
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
tot = sum(sum(v) for v in agg.values())
for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    extra = f" {sum(v)/steps/1e3:7.3f} ms/step" if steps else ""
    print(f"{len(v):6d} {sum(v)/1e3:9.2f}ms avg {sum(v)/len(v):8.1f}us max {max(v):8.1f}us {100*sum(v)/tot:5.1f}%{extra}  {n}")
