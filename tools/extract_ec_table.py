"""Extract the fixed-base tables of EllipicCurveScalarGeneratorMult for the implemented curves.

Source: the reference's ec/powers/<curve>pows.circom (get_g_pow_stride8_table_<curve>, 32 x 256 x 2 x 4
64-bit limbs: powers[i][j] = j * 2^(8 i) * G, limbs little-endian; powers[i][0] = 0), read as text.
Every entry is checked against an independent affine computation of j * 2^(8 i) * G (curve
parameters from FIPS 186-4 / RFC 5639, pzkwit/inputs.py) before the binary is written, so each
committed data file is pinned both to the reference text and to the curve arithmetic.

Output: passport-zk-circuits_amd/data/<p256|bp256>_gpow8.bin = 32*256*2*4 little-endian u64 (512 KiB).
Run (in the build container, where /root/reference exists):
    python tools/extract_ec_table.py p256|bp256
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "passport-zk-circuits_amd"))
from pzkwit.inputs import BP256, P256  # noqa: E402

POWERS = "/root/reference/circuits/lib/circuits/ec/powers/"
CURVES = {"p256": (P256, POWERS + "p256pows.circom"), "bp256": (BP256, POWERS + "brainpoolP256r1pows.circom")}


def expected_table(curve):
    t = np.zeros((32, 256, 2, 4), dtype=np.uint64)
    base = curve.g
    for i in range(32):
        acc = None
        for j in range(1, 256):
            acc = curve.add(acc, base)
            for a, v in enumerate(acc):
                for k in range(4):
                    t[i, j, a, k] = (v >> (64 * k)) & (2 ** 64 - 1)
        for _ in range(8):
            base = curve.add(base, base)
    return t


def parse(path):
    t = np.zeros((32, 256, 2, 4), dtype=np.uint64)
    seen = np.zeros((32, 256, 2, 4), dtype=bool)
    pat = re.compile(r"powers\[(\d+)\]\[(\d+)\]\[(\d+)\]\[(\d+)\]\s*=\s*(\d+);")
    with open(path) as f:
        for line in f:
            m = pat.search(line)
            if m:
                i, j, a, k, v = (int(x) for x in m.groups())
                t[i, j, a, k] = v
                seen[i, j, a, k] = True
    if not seen.all():
        raise SystemExit("table incomplete: %d of %d entries" % (seen.sum(), seen.size))
    return t


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "p256"
    curve, src = CURVES[name]
    ref = parse(sys.argv[2] if len(sys.argv) > 2 else src)
    exp = expected_table(curve)
    bad = np.argwhere(ref != exp)
    if bad.size:
        raise SystemExit("reference table differs from j*2^(8i)*G at %s" % (bad[:4].tolist(),))
    out = os.path.join(HERE, "..", "passport-zk-circuits_amd", "data", "%s_gpow8.bin" % name)
    ref.astype("<u8").tofile(out)
    print("wrote %s (%d bytes), all %d entries = j*2^(8i)*G" % (out, ref.nbytes, ref.size // 8))


if __name__ == "__main__":
    main()
