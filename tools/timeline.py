"""Print the kernel timeline of the last batch from a rocprofv3 kernel-trace CSV."""
import csv
import sys


def main(path, marker="k_load_values", which=-1):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    s = idx[which]
    e = idx[which + 1] if which + 1 < 0 or which + 1 < len(idx) and which != -1 else len(rows)
    t0 = int(rows[s]["Start_Timestamp"])
    for r in rows[s:e]:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pzk::", "")
        a, b = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{n:30s} q={r.get('Queue_Id', ''):2s} {a / 1e6:8.2f} {b / 1e6:8.2f} {(b - a) / 1e6:7.2f}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
