"""Independent pure-Python restatements of the public-output formulas, used by the tests to
pin values the circuit exports (no circom code is evaluated here):

* BabyJubJub scalar multiplication by Base8 — twisted Edwards a*x^2 + y^2 = 1 + d*x^2*y^2,
  a = 168700, d = 168696 (babyjubjub/curve.circom:62-105, get.circom:9-10); affine addition
  law x3 = (x1 y2 + y1 x2)/(1 + d x1 x2 y1 y2), y3 = (y1 y2 - a x1 x2)/(1 - d x1 x2 y1 y2).
* dg1Commitment = Poseidon5(4 x Bits2Num(186) of DG1 bits, Poseidon1(sk)) (identity.circom:89-109;
  the same formula helpers/generateRegisterIdentityTest.js:187-201 re-derives with @iden3/js-crypto).
* dg15PubKeyHash for an RSA-1024 AA key = Poseidon5(200,200,200,200,224-bit chunks) (README.md:72-75).
"""
from pzkwit.field import P, poseidon
from pzkwit.inputs import bits_msb_first, sha_pad

A, D = 168700, 168696
B8 = (5299619240641551281634865583518297030282874472190772894086521144482721001553,
      16950150798460657717958625567821834550301663161624707787222815936182638968203)


def bjj_add(p1, p2):
    (x1, y1), (x2, y2) = p1, p2
    t = D * x1 * x2 * y1 * y2 % P
    x3 = (x1 * y2 + y1 * x2) * pow(1 + t, -1, P) % P
    y3 = (y1 * y2 - A * x1 * x2) * pow(1 - t, -1, P) % P
    return x3, y3


def bjj_mul(k, base=B8):
    r = (0, 1)  # group identity
    for i in reversed(range(k.bit_length())):
        r = bjj_add(r, r)
        if (k >> i) & 1:
            r = bjj_add(r, base)
    return r


def dg1_commitment(dg1_bytes, sk, chunk=186):
    bits = [int(b) for b in bits_msb_first(sha_pad(dg1_bytes, 512))]
    nums = [sum(bits[i * chunk + j] << j for j in range(chunk)) for i in range(4)]
    return poseidon(nums + [poseidon([sk])])


def aa_rsa_hash(dg15_bytes, aa_shift_bits):
    bits = [int(b) for b in bits_msb_first(sha_pad(dg15_bytes, 512))]
    chunks = []
    for j in range(5):
        ln = 200 if j < 4 else 224
        seg = bits[aa_shift_bits + 200 * j: aa_shift_bits + 200 * j + ln]
        chunks.append(int("".join(map(str, seg)), 2))
    return poseidon(chunks)
