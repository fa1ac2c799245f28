"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` remarks: one line per kernel."""
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def main(path):
    rows, cur = [], None
    for line in open(path):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"LDS Size \[bytes/block\]|VGPRs Spill|SGPRs Spill): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).split(" [")[0]] = int(m.group(2))
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        n = re.sub(r"\(.*", "", n).replace("pzk::", "")
        print(f"{n:34s} vgpr={r.get('VGPRs',0):3d} agpr={r.get('AGPRs',0):3d} sgpr={r.get('TotalSGPRs',0):3d} "
              f"scratch={r.get('ScratchSize',0):5d} occ={r.get('Occupancy',0)} lds={r.get('LDS Size',0)} "
              f"vspill={r.get('VGPRs Spill',0)}")


if __name__ == "__main__":
    main(sys.argv[1])
