"""Per-kernel private segment (scratch bytes per lane) of the built gfx950 code objects.

Scratch on this path is never intended: a private array indexed at run time (or a loop the compiler did not
unroll over a register array) is lowered to scratch, and under the emitters' store stream its lines reach
HBM (k_emit_gen's 272 B per lane doubled that kernel's traffic). Usage: python tools/kernel_scratch.py [--all]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
BUILD = os.path.join(os.path.dirname(__file__), "..", "passport-zk-circuits_amd", "csrc", "build")


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        local = os.path.join(d, os.path.basename(obj))
        subprocess.run(["cp", obj, local], check=True)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", local], cwd=d, capture_output=True)
        co = [f for f in os.listdir(d) if "gfx950" in f]
        if not co:
            return []
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(d, co[0])], capture_output=True,
                               text=True).stdout
    out, name = [], None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name:
            out.append((name, int(m.group(1))))
    return out


def main():
    show_all = "--all" in sys.argv
    rows = []
    for obj in sorted(glob.glob(os.path.join(BUILD, "*.hip.o"))):
        for name, sz in kernels(obj):
            if sz or show_all:
                rows.append((sz, os.path.basename(obj), name))
    names = subprocess.run(["c++filt"], input="\n".join(r[2] for r in rows), capture_output=True,
                           text=True).stdout.splitlines() if rows else []
    for (sz, obj, _), n in sorted(zip(rows, names), key=lambda x: -x[0][0]):
        print(f"{sz:6d}  {obj:24s} {re.sub(r'[(].*', '', n).replace('pzk::', '')}")


if __name__ == "__main__":
    main()
