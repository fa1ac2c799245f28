"""Regenerate the fixed-base tables of EllipicCurveScalarGeneratorMult (ec/curve.circom:672-735).

The reference includes one table per curve, `get_g_pow_stride8_table_<curve>(n, k)` in
ec/powers/<curve>pows.circom: powers[i][j][axis][chunk] = chunk `chunk` (n bits, little-endian) of
coordinate `axis` of j * 2^(8 i) * G, for i < n * k / 8 and j < 256, with powers[i][0] = (0, 0). Six of the
eleven files are missing from the snapshot (.MISSING_LARGE_BLOBS: brainpoolP320r1, brainpoolP384r1,
brainpoolP512r1, p384, secp192r1, secp521r1). They are deterministic, so this script computes them:

  1. for every curve whose file IS present (p256, secp256k1, brainpoolP256r1, secp224r1, brainpoolP224r1) it
     writes the whole .circom text and compares it with the reference file BYTE FOR BYTE — which pins the
     text format and the generator / chunking of each of those curves;
  2. every curve's parameters are checked against the reference's own constants: A, B, P against
     signatureVerification.circom (SIGNATURE_TYPE 20-25), the order and the dummy point against
     EllipicCurveGetOrder / EllipticCurveGetDummy (ec/get.circom:79-195): G lies on the curve, order * G is
     the point at infinity, and the dummy point is 2^m * G for the m the reference used;
  3. the same code then writes the missing curves' tables (text under --out-circom if asked) and the binary
     tables the GPU path and the CPU oracle load: passport-zk-circuits_amd/data/<name>_gpow8.bin =
     parts x 256 x 2 x k little-endian u64 chunks.

Curve parameters: FIPS 186-4 D.1.2 (P-192, P-224, P-256, P-384), SEC 2 2.4.1 (secp256k1), RFC 5639 3.2-3.6
(brainpool). Run in the build container (reads /root/reference):
    python tools/gen_ec_tables.py [--out-circom DIR]
"""
import argparse
import hashlib
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/circuits"
POWERS = REF + "/lib/circuits/ec/powers/"
DATA = os.path.join(HERE, "..", "passport-zk-circuits_amd", "data")


def H(s):
    return int(s, 16)


# name: (p, a, b, gx, gy, n, chunk bits, chunks, SIGNATURE_TYPE using it or None, data file stem or None)
CURVES = {
    "p256": (H("FFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF"), -3,
             H("5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B"),
             H("6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296"),
             H("4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5"),
             H("FFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551"), 64, 4, 20, "p256"),
    "secp256k1": (H("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F"), 0, 7,
                  H("79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798"),
                  H("483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8"),
                  H("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141"), 64, 4, None, None),
    "brainpoolP256r1": (H("A9FB57DBA1EEA9BC3E660A909D838D726E3BF623D52620282013481D1F6E5377"),
                        H("7D5A0975FC2C3057EEF67530417AFFE7FB8055C126DC5C6CE94A4B44F330B5D9"),
                        H("26DC5C6CE94A4B44F330B5D9BBD77CBF958416295CF7E1CE6BCCDC18FF8C07B6"),
                        H("8BD2AEB9CB7E57CB2C4B482FFC81B7AFB9DE27E1E3BD23C23A4453BD9ACE3262"),
                        H("547EF835C3DAC4FD97F8461A14611DC9C27745132DED8E545C1D54C72F046997"),
                        H("A9FB57DBA1EEA9BC3E660A909D838D718C397AA3B561A6F7901E0E82974856A7"), 64, 4, 21, "bp256"),
    "secp224r1": (H("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF000000000000000000000001"), -3,
                  H("B4050A850C04B3ABF54132565044B0B7D7BFD8BA270B39432355FFB4"),
                  H("B70E0CBD6BB4BF7F321390B94A03C1D356C21122343280D6115C1D21"),
                  H("BD376388B5F723FB4C22DFE6CD4375A05A07476444D5819985007E34"),
                  H("FFFFFFFFFFFFFFFFFFFFFFFFFFFF16A2E0B8F03E13DD29455C5C2A3D"), 32, 7, 24, "p224"),
    "brainpoolP224r1": (H("D7C134AA264366862A18302575D1D787B09F075797DA89F57EC8C0FF"),
                        H("68A5E62CA9CE6C1C299803A6C1530B514E182AD8B0042A59CAD29F43"),
                        H("2580F63CCFE44138870713B1A92369E33E2135D266DBB372386C400B"),
                        H("0D9029AD2C7E5CF4340823B2A87DC68C9E4CE3174C1E6EFDEE12C07D"),
                        H("58AA56F772C0726F24C6B89E4ECDAC24354B9E99CAA3F6D3761402CD"),
                        H("D7C134AA264366862A18302575D0FB98D116BC4B6DDEBCA3A5A7939F"), 32, 7, None, None),
    "brainpoolP320r1": (H("D35E472036BC4FB7E13C785ED201E065F98FCFA6F6F40DEF4F92B9EC7893EC28FCD412B1F1B32E27"),
                        H("3EE30B568FBAB0F883CCEBD46D3F3BB8A2A73513F5EB79DA66190EB085FFA9F492F375A97D860EB4"),
                        H("520883949DFDBC42D3AD198640688A6FE13F41349554B49ACC31DCCD884539816F5EB4AC8FB1F1A6"),
                        H("43BD7E9AFB53D8B85289BCC48EE5BFE6F20137D10A087EB6E7871E2A10A599C710AF8D0D39E20611"),
                        H("14FDD05545EC1CC8AB4093247F77275E0743FFED117182EAA9C77877AAAC6AC7D35245D1692E8EE1"),
                        H("D35E472036BC4FB7E13C785ED201E065F98FCFA5B68F12A32D482EC7EE8658E98691555B44C59311"),
                        64, 5, 22, None),
    "brainpoolP384r1": (H("8CB91E82A3386D280F5D6F7E50E641DF152F7109ED5456B412B1DA197FB71123ACD3A729901D1A71874700133107EC53"),
                        H("7BC382C63D8C150C3C72080ACE05AFA0C2BEA28E4FB22787139165EFBA91F90F8AA5814A503AD4EB04A8C7DD22CE2826"),
                        H("04A8C7DD22CE28268B39B55416F0447C2FB77DE107DCD2A62E880EA53EEB62D57CB4390295DBC9943AB78696FA504C11"),
                        H("1D1C64F068CF45FFA2A63A81B7C13F6B8847A3E77EF14FE3DB7FCAFE0CBD10E8E826E03436D646AAEF87B2E247D4AF1E"),
                        H("8ABE1D7520F9C2A45CB1EB8E95CFD55262B70B29FEEC5864E19C054FF99129280E4646217791811142820341263C5315"),
                        H("8CB91E82A3386D280F5D6F7E50E641DF152F7109ED5456B31F166E6CAC0425A7CF3AB6AF6B7FC3103B883202E9046565"),
                        64, 6, 25, "bp384"),
    "p384": (H("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFFFF0000000000000000FFFFFFFF"), -3,
             H("B3312FA7E23EE7E4988E056BE3F82D19181D9C6EFE8141120314088F5013875AC656398D8A2ED19D2A85C8EDD3EC2AEF"),
             H("AA87CA22BE8B05378EB1C71EF320AD746E1D3B628BA79B9859F741E082542A385502F25DBF55296C3A545E3872760AB7"),
             H("3617DE4A96262C6F5D9E98BF9292DC29F8F41DBD289A147CE9DA3113B5F0B8C00A60B1CE1D7E819D7A431D7C90EA0E5F"),
             H("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFC7634D81F4372DDF581A0DB248B0A77AECEC196ACCC52973"),
             64, 6, None, None),
    "secp192r1": (H("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFFFFFFFFFFFF"), -3,
                  H("64210519E59C80E70FA7E9AB72243049FEB8DEECC146B9B1"),
                  H("188DA80EB03090F67CBF20EB43A18800F4FF0AFD82FF1012"),
                  H("07192B95FFC8DA78631011ED6B24CDD573F977A11E794811"),
                  H("FFFFFFFFFFFFFFFFFFFFFFFF99DEF836146BC9B1B4D22831"), 64, 3, 23, None),
}


class Curve:
    def __init__(self, p, a, b, gx, gy, n):
        self.p, self.a, self.b, self.g, self.n = p, a % p, b % p, (gx, gy), n

    def on_curve(self, pt):
        x, y = pt
        return (y * y - (x * x * x + self.a * x + self.b)) % self.p == 0

    def add(self, p1, p2):
        if p1 is None:
            return p2
        if p2 is None:
            return p1
        P = self.p
        (x1, y1), (x2, y2) = p1, p2
        if x1 == x2:
            if (y1 + y2) % P == 0:
                return None
            lam = (3 * x1 * x1 + self.a) * pow(2 * y1, -1, P) % P
        else:
            lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
        x3 = (lam * lam - x1 - x2) % P
        return x3, (lam * (x1 - x3) - y1) % P

    def mul(self, k, pt=None):
        pt = self.g if pt is None else pt
        r = None
        for i in reversed(range(k.bit_length())):
            r = self.add(r, r)
            if (k >> i) & 1:
                r = self.add(r, pt)
        return r


def chunks(v, n, k):
    return [(v >> (n * i)) & ((1 << n) - 1) for i in range(k)]


def table(name):
    """powers[i][j][axis][chunk] as an int array [parts][256][2][k] (object dtype: chunks up to 64 bits)"""
    p, a, b, gx, gy, order, n, k, _, _ = CURVES[name]
    c = Curve(p, a, b, gx, gy, order)
    parts = n * k // 8
    t = np.zeros((parts, 256, 2, k), dtype=np.uint64)
    base = c.g
    for i in range(parts):
        acc = None
        for j in range(1, 256):
            acc = c.add(acc, base)
            for ax in range(2):
                t[i, j, ax] = chunks(acc[ax], n, k)
        for _ in range(8):
            base = c.add(base, base)
    return t


def circom_text(name, t):
    n, k = CURVES[name][6], CURVES[name][7]
    parts = t.shape[0]
    out = ["pragma circom 2.1.6;\n\nfunction get_g_pow_stride8_table_%s(n, k) {\n" % name,
           "    assert(n == %d && k == %d);\n" % (n, k), "    var powers[%d][256][2][%d];\n\n" % (parts, k)]
    for i in range(parts):
        for j in range(256):
            for ax in range(2):
                for q in range(k):
                    out.append("    powers[%d][%d][%d][%d] = %d;\n" % (i, j, ax, q, int(t[i, j, ax, q])))
            out.append("\n")
    out.append("    return powers;\n}\n")
    return "".join(out)


def ref_limbs(text, pattern):
    m = re.search(pattern, text, re.S)
    return [int(x) for x in re.findall(r"\d+", m.group(1))] if m else None


def to_int(limbs, n):
    return sum(v << (n * i) for i, v in enumerate(limbs))


def check_params(name):
    """the curve's constants against the reference's: A/B/P (signatureVerification.circom), order and dummy
    (get.circom, found by P); G on the curve, order * G = infinity, dummy = 2^m * G. Returns notes."""
    p, a, b, gx, gy, order, n, k, sig, _ = CURVES[name]
    c = Curve(p, a, b, gx, gy, order)
    notes = []
    assert c.on_curve(c.g), name + ": G not on the curve"
    assert c.mul(order) is None, name + ": order * G != infinity"
    plimbs = chunks(p, n, k)
    if sig is not None:
        sv = open(REF + "/signatureVerifier/signatureVerification.circom").read()
        blk = sv[sv.index("if (SIG_ALGO == %d){" % sig, sv.index("component ")):]
        arrs = [[int(x) for x in re.findall(r"\d+", a_)] for a_ in re.findall(r"\[([\d,\s]+)\]", blk)[:3]]
        assert arrs[0] == chunks(a % p, n, k), name + ": A differs from signatureVerification.circom"
        assert arrs[1] == chunks(b, n, k), name + ": B differs"
        assert arrs[2] == plimbs, name + ": P differs"
        notes.append("A/B/P = signatureVerification.circom SIG %d" % sig)
    gt = open(REF + "/lib/circuits/ec/get.circom").read()
    pcond = " && ".join("P[%d] == %d" % (i, v) for i, v in enumerate(plimbs))
    for tmpl, key in (("EllipicCurveGetOrder", "order"), ("EllipticCurveGetDummy", "dummy")):
        body = gt[gt.index("template " + tmpl):]
        at = body.find(pcond)
        if at < 0:
            continue
        seg = body[at:body.index("}", at)]
        arrs = [[int(x) for x in re.findall(r"\d+", a_)] for a_ in re.findall(r"<==\s*\[([\d,\s]+)\]", seg)]
        if key == "order":
            assert to_int(arrs[0], n) == order, name + ": order differs from get.circom"
            notes.append("order = get.circom")
        else:
            d = (to_int(arrs[0], n), to_int(arrs[1], n))
            assert c.on_curve(d), name + ": get.circom dummy not on the curve"
            pt, m = c.g, 0
            while pt != d and m < 1024:
                pt, m = c.add(pt, pt), m + 1
            assert pt == d, name + ": dummy is not 2^m G"
            notes.append("dummy = 2^%d G (get.circom)" % m)
    return notes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-circom", default=None, help="also write <curve>pows.circom of the missing curves here")
    args = ap.parse_args()
    for name, spec in CURVES.items():
        notes = check_params(name)
        t = table(name)
        text = circom_text(name, t)
        ref = POWERS + "%spows.circom" % name
        digest = hashlib.sha256(text.encode()).hexdigest()[:16]
        if os.path.exists(ref):
            same = open(ref, "rb").read() == text.encode()
            assert same, name + ": generated text differs from " + ref
            notes.append("text == reference file byte for byte (%d bytes, sha256 %s)" % (len(text), digest))
        else:
            notes.append("reference file missing from the snapshot: generated (%d bytes, sha256 %s)" % (len(text), digest))
            if args.out_circom:
                os.makedirs(args.out_circom, exist_ok=True)
                open(os.path.join(args.out_circom, "%spows.circom" % name), "w").write(text)
        if spec[9]:
            out = os.path.join(DATA, "%s_gpow8.bin" % spec[9])
            t.astype("<u8").tofile(out)
            notes.append("wrote data/%s_gpow8.bin (%d bytes)" % (spec[9], t.nbytes))
        print("%-16s %s" % (name, "; ".join(notes)))


if __name__ == "__main__":
    main()
