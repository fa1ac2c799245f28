"""Extract the P-256 fixed-base table of EllipicCurveScalarGeneratorMult.

Source: the reference's ec/powers/p256pows.circom (get_g_pow_stride8_table_p256, 32 x 256 x 2 x 4
64-bit limbs: powers[i][j] = j * 2^(8 i) * G, limbs little-endian; powers[i][0] = 0), read as text.
Every entry is checked against an independent affine computation of j * 2^(8 i) * G before the
binary is written, so the committed data file is pinned both to the reference text and to the
curve arithmetic.

Output: passport-zk-circuits_amd/data/p256_gpow8.bin = 32*256*2*4 little-endian u64 (512 KiB).
Run (in the build container, where /root/reference exists):
    python tools/extract_p256_table.py [/root/reference/circuits/lib/circuits/ec/powers/p256pows.circom]
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "passport-zk-circuits_amd", "data", "p256_gpow8.bin")
SRC = "/root/reference/circuits/lib/circuits/ec/powers/p256pows.circom"

# secp256r1 (FIPS 186-4 D.1.2.3)
P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
A = P - 3
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5


def ec_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 + A) * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def expected_table():
    t = np.zeros((32, 256, 2, 4), dtype=np.uint64)
    base = (GX, GY)
    for i in range(32):
        acc = None
        for j in range(1, 256):
            acc = ec_add(acc, base)
            for a, v in enumerate(acc):
                for k in range(4):
                    t[i, j, a, k] = (v >> (64 * k)) & (2 ** 64 - 1)
        for _ in range(8):
            base = ec_add(base, base)
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
    src = sys.argv[1] if len(sys.argv) > 1 else SRC
    ref = parse(src)
    exp = expected_table()
    bad = np.argwhere(ref != exp)
    if bad.size:
        raise SystemExit("reference table differs from j*2^(8i)*G at %s" % (bad[:4].tolist(),))
    ref.astype("<u8").tofile(OUT)
    print("wrote %s (%d bytes), all %d entries = j*2^(8i)*G" % (OUT, ref.nbytes, ref.size // 8))


if __name__ == "__main__":
    main()
