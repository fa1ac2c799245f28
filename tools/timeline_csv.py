"""Per-kernel timeline (ms, relative) of one window of a rocprofv3 --kernel-trace CSV:
python tools/timeline_csv.py run_kernel_trace.csv [anchor_substring] [nth] [count]"""
import csv
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_load_values"
nth = int(sys.argv[3]) if len(sys.argv) > 3 else -1
count = int(sys.argv[4]) if len(sys.argv) > 4 else 40
rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
               for r in csv.DictReader(open(path))), key=lambda r: r[1])
idx = [i for i, r in enumerate(rows) if anchor in r[0]]
i0 = idx[nth]
t0 = rows[i0][1]
for name, s, e, q in rows[i0:i0 + count]:
    short = name.split("(")[0].replace("void ", "").replace("pzk::", "")
    print("%-32s q=%-3s %8.2f %8.2f %7.2f" % (short[:32], q, (s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6))
