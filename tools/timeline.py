"""Print a per-kernel timeline (ms, relative) of one window of a rocprofv3 rocpd database:
python tools/timeline.py DB [first_kernel_substring] [nth] [count]"""
import sqlite3
import sys

db = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_load_values"
nth = int(sys.argv[3]) if len(sys.argv) > 3 else -1
count = int(sys.argv[4]) if len(sys.argv) > 4 else 40
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
rows = list(c.execute("select name, start, end, queue_id from kernels order by start"))
idx = [i for i, r in enumerate(rows) if anchor in r[0]]
i0 = idx[nth]
t0 = rows[i0][1]
for name, s, e, q in rows[i0:i0 + count]:
    short = name.split("(")[0].replace("void ", "").replace("pzk::", "")
    print("%-32s q=%-3s %8.2f %8.2f %7.2f" % (short[:32], q, (s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6))
