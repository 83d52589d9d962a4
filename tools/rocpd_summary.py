"""Per-kernel duration summary (median / min per kernel name and grid) of a rocprofv3 rocpd database: python tools/rocpd_summary.py <results.db>."""
import sqlite3,sys,collections
c=sqlite3.connect(sys.argv[1])
d=collections.defaultdict(list)
for name,dur,gx in c.execute("select name,duration,grid_x from kernels"):
    d[(name[:80],gx)].append(dur/1e3)
for k,v in sorted(d.items(), key=lambda kv:-sum(kv[1])):
    v.sort(); print(f"{k[0]:80s} grid={k[1]:8d} n={len(v):3d} med={v[len(v)//2]:9.1f}us min={v[0]:9.1f}")
