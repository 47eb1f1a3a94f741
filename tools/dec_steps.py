"""Per-step decode kernel times from a rocprofv3 kernel trace (rocpd .db): the last query's
batches, grouped in lock steps (pred<0>, pred<1>, G, joint).  Development tool.
    python tools/dec_steps.py gpurun_out/<dir>"""
import glob
import sqlite3
import sys

import numpy as np

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, grid_x/workgroup_x from kernels order by start").fetchall()
jt = [i for i, r in enumerate(rows) if "joint_trans" in r[0]]
names = ["pred_kernel<0", "pred_kernel<1", "dec_g", "dec_joint"]
for b in range(3):
    s = jt[-3 + b]
    e = jt[-3 + b + 1] if b < 2 else len(rows)
    dec = [r for r in rows[s:e] if any(n in r[0] for n in names)]
    steps, cur = [], {}
    for r in dec:
        k = [n for n in names if n in r[0]][0]
        cur[k] = (r[2] - r[1]) / 1e3
        if k == "dec_joint":
            steps.append(cur)
            cur = {}
    st = np.array([[x.get(n, 0) for n in names] for x in steps])
    span = (dec[-1][2] - dec[0][1]) / 1e6
    print(f"batch {b}: steps {len(st)}, span {span:.1f} ms, kernel sum {st.sum() / 1e3:.1f} ms, "
          f"per-kernel mean {st.mean(0).round(1)}")
    for lo, hi in [(0, 50), (50, 100), (100, 200), (200, 300), (300, 400), (400, 600), (600, 900)]:
        m = st[lo:hi]
        if len(m):
            print(f"   steps {lo}-{hi}: mean per step {m.sum(1).mean():.1f} us  {m.mean(0).round(1)}")
