"""QueryIdentity(80) inputs (identityManagement/queryIdentity.circom:37-229): the input row layout, the
JSON signal names of the circuit, and a deterministic generator of valid synthetic queries (a TD3 DG1 with
real MRZ field positions, an identity-state Sparse Merkle Tree proof of chosen depth, bounds that the
selected checks accept), used by the tests and by `bench.py --workload query`.

Row layout = main's input declaration order (842 elements of 32 B, little-endian, normal form):
eventID, eventData, idStateRoot, selector, currentDate, timestampLowerbound, timestampUpperbound,
identityCounterLowerbound, identityCounterUpperbound, birthDateLowerbound, birthDateUpperbound,
expirationDateLowerbound, expirationDateUpperbound, citizenshipMask, skIdentity, pkPassportHash, dg1[744],
idStateSiblings[80], timestamp, identityCounter.
"""
import os

import numpy as np

from .field import P, SplitMix64, poseidon

NAMES = ["eventID", "eventData", "idStateRoot", "selector", "currentDate", "timestampLowerbound",
         "timestampUpperbound", "identityCounterLowerbound", "identityCounterUpperbound", "birthDateLowerbound",
         "birthDateUpperbound", "expirationDateLowerbound", "expirationDateUpperbound", "citizenshipMask",
         "skIdentity", "pkPassportHash", "dg1", "idStateSiblings", "timestamp", "identityCounter"]
LENGTHS = {"dg1": 744, "idStateSiblings": 80}
N_INPUTS = 842
DEPTH = 80
# QueryIdentityTD1 (queryIdentityTD1.circom): dg1[760], the rest identical
LENGTHS_TD1 = {"dg1": 760, "idStateSiblings": 80}
N_INPUTS_TD1 = 858


def _offsets(lengths):
    off, o = {}, 0
    for n in NAMES:
        off[n] = o
        o += lengths.get(n, 1)
    return off, o


OFF, _n3 = _offsets(LENGTHS)
OFF_TD1, _n1 = _offsets(LENGTHS_TD1)
assert _n3 == N_INPUTS and _n1 == N_INPUTS_TD1

# CitizenshipCheck COUNTRY_ARR (data/citizenship_codes.inc, extracted from citizenshipCheck.circom)
_INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "citizenship_codes.inc")


def countries():
    vals = []
    for line in open(_INC):
        line = line.split("/*")[0]
        if not line.strip() or line.lstrip().startswith("*"):
            continue
        vals += [int(t.strip().rstrip("u")) for t in line.split(",") if t.strip()]
    assert len(vals) == 240
    return vals


# BabyJubJub (twisted Edwards a x^2 + y^2 = 1 + d x^2 y^2), Base8 (babyjubjub/get.circom)
A_BJJ, D_BJJ = 168700, 168696
BASE8 = (5299619240641551281634865583518297030282874472190772894086521144482721001553,
         16950150798460657717958625567821834550301663161624707787222815936182638968203)


def bjj_add(p1, p2):
    (x1, y1), (x2, y2) = p1, p2
    t = D_BJJ * x1 * x2 * y1 * y2 % P
    return ((x1 * y2 + y1 * x2) * pow(1 + t, -1, P) % P, (y1 * y2 - A_BJJ * x1 * x2) * pow(1 - t, -1, P) % P)


def bjj_mul(k, base=BASE8):
    r = (0, 1)
    for i in reversed(range(k.bit_length())):
        r = bjj_add(r, r)
        if (k >> i) & 1:
            r = bjj_add(r, base)
    return r


def enc_date(yy, mm, dd):
    """(YY, MM, DD) -> the circuit's encoded date: UTF-8 "YYMMDD" read big-endian."""
    return int.from_bytes(b"%02d%02d%02d" % (yy, mm, dd), "big")


def smt_root(key, value, siblings):
    """Root of an iden3 SMT proof (SMTVerifier.circom): the leaf SMTHash1(key, value) = Poseidon3(key, value, 1)
    at the insertion level j (siblings[j:] zero), then level hashes Poseidon2(L, R) up to the root with the
    key's bit i choosing the side."""
    j = len(siblings)
    while j > 0 and siblings[j - 1] == 0:
        j -= 1
    child = poseidon([key, value, 1])
    for i in range(j - 1, -1, -1):
        if (key >> i) & 1:
            child = poseidon([siblings[i], child])
        else:
            child = poseidon([child, siblings[i]])
    return child


_MRZ = b"ABCDEFGHIJKLMNOPQRSTUVWXYZ<"


def make_query(rng, depth=None, selector=None, cit_code=None, td1=False, **over):
    """One valid query: -> (inputs dict of python ints / lists, info dict). `over` replaces inputs after
    generation (the SMT root is NOT recomputed for them); cit_code: a 3-byte issuing-state code for the DG1
    (the identity state is built over that DG1); td1: a TD1 (ID card) DG1 for QueryIdentityTD1."""
    C = countries()
    cidx = rng.below(240)
    cit = C[cidx].to_bytes(3, "big") if cit_code is None else cit_code
    nat = C[rng.below(240)].to_bytes(3, "big")
    by, bm, bd = (50 + rng.below(50)) if rng.below(4) else rng.below(20), 1 + rng.below(12), 1 + rng.below(28)
    ey, em, ed = 25 + rng.below(10), 1 + rng.below(12), 1 + rng.below(28)
    name = bytes(_MRZ[rng.below(len(_MRZ))] for _ in range(39))
    docnum = bytes(b"0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ"[rng.below(36)] for _ in range(9))
    sex = b"MF<"[rng.below(3):][:1]
    if not td1:
        line1 = b"P<" + cit + name
        line2 = (docnum + b"0" + nat + b"%02d%02d%02d" % (by, bm, bd) + b"0" + sex + b"%02d%02d%02d" % (ey, em, ed) +
                 b"0" + b"<" * 14 + b"00")
        assert len(line1) == 44 and len(line2) == 44
        dg1 = bytes.fromhex("615b5f1f58") + line1 + line2
    else:  # TD1: 3 x 30 MRZ characters (ICAO 9303-5): type, state, number, optional data | dates, sex, nationality | name
        pers = bytes(b"0123456789"[rng.below(10)] for _ in range(11))
        l1 = b"ID" + cit + docnum + b"0" + pers + b"<" * 4
        l2 = b"%02d%02d%02d" % (by, bm, bd) + b"0" + sex + b"%02d%02d%02d" % (ey, em, ed) + b"0" + nat + b"<" * 11 + b"0"
        l3 = name[:30]
        assert len(l1) == 30 and len(l2) == 30 and len(l3) == 30
        dg1 = bytes.fromhex("615d5f1f5a") + l1 + l2 + l3
    bits = np.unpackbits(np.frombuffer(dg1, dtype=np.uint8)).astype(int).tolist()
    assert len(bits) == (760 if td1 else 744)
    sk = rng.fr() >> 2
    pk_pass = rng.fr()
    ts = 1_700_000_000 + rng.below(100_000_000)
    ic = rng.below(1000)
    # identity state: value = Poseidon3(dgCommit, counter, timestamp), key = Poseidon2(pkPassHash, pkIdentityHash)
    ch = 190 if td1 else 186
    chunks = [int("".join(map(str, bits[ch * i:ch * (i + 1)]))[::-1] or "0", 2) for i in range(4)]
    sk_h = poseidon([sk])
    dg_commit = poseidon(chunks + [sk_h])
    ax, ay = bjj_mul(sk)
    key = poseidon([pk_pass, poseidon([ax, ay])])
    value = poseidon([dg_commit, ic, ts])
    d = rng.below(DEPTH) if depth is None else depth
    sib = [rng.fr() or 1 for _ in range(d)] + [0] * (DEPTH - d)
    root = smt_root(key, value, sib)
    mask = rng.bits(240) & ~(1 << (239 - cidx))
    sel = rng.bits(18) if selector is None else selector
    cur = enc_date(24, 10, 17)
    inp = {
        "eventID": rng.fr(), "eventData": rng.fr(), "idStateRoot": root, "selector": sel, "currentDate": cur,
        "timestampLowerbound": ts - rng.below(1000), "timestampUpperbound": ts + 1 + rng.below(1000),
        "identityCounterLowerbound": ic - rng.below(ic + 1), "identityCounterUpperbound": ic + 1 + rng.below(10),
        "birthDateLowerbound": enc_date(30, 1 + rng.below(12), 1 + rng.below(28)),
        "birthDateUpperbound": enc_date(20 + rng.below(4), 1 + rng.below(12), 1 + rng.below(28)),
        "expirationDateLowerbound": enc_date(ey - 1, 1 + rng.below(12), 1 + rng.below(28)),
        "expirationDateUpperbound": enc_date(ey + 1, 1 + rng.below(12), 1 + rng.below(28)),
        "citizenshipMask": mask, "skIdentity": sk, "pkPassportHash": pk_pass, "dg1": bits, "idStateSiblings": sib,
        "timestamp": ts, "identityCounter": ic,
    }
    inp.update(over)
    spec = (((280, 48), (344, 48), (520, 240), (400, 24), (56, 24), (336, 8), (80, 72), (160, 88), (40, 16)) if td1 else
            ((496, 48), (560, 48), (80, 248), (328, 64), (472, 24), (56, 24), (552, 8), (392, 72)))
    fields = [int.from_bytes(dg1[o // 8:o // 8 + n // 8], "big") for o, n in spec]
    info = {"fields": fields, "nullifier": poseidon([sk, sk_h, inp["eventID"]]), "dg_commit": dg_commit,
            "pk_identity": (ax, ay), "key": key, "value": value, "depth": d, "citizenship_index": cidx, "td1": td1}
    return inp, info


def pack(inp, out=None):
    """inputs dict -> (842 | 858 (TD1), 32) uint8 row (normal form, little-endian)."""
    td1 = len(inp["dg1"]) == 760
    lengths, off = (LENGTHS_TD1, OFF_TD1) if td1 else (LENGTHS, OFF)
    row = out if out is not None else np.zeros((N_INPUTS_TD1 if td1 else N_INPUTS, 32), dtype=np.uint8)
    for name in NAMES:
        v = inp[name]
        vals = v if isinstance(v, (list, tuple)) else [v]
        assert len(vals) == lengths.get(name, 1), name
        for i, x in enumerate(vals):
            row[off[name] + i] = np.frombuffer((int(x) % P).to_bytes(32, "little"), dtype=np.uint8)
    return row


def public_outputs(inp, info):
    """Main outputs [nullifier, birthDate, expirationDate, name, nameResidual, nationality, citizenship, sex,
    documentNumber] (TD1: [nullifier, birthDate, expirationDate, name, nationality, citizenship, sex,
    Poseidon1(documentNumber), Poseidon1(personalNumber), documentType]), each masked by its selector bit
    (queryIdentity.circom:86-105, queryIdentityTD1.circom:97-105)."""
    sel = inp["selector"]
    bit = lambda k: (sel >> k) & 1  # noqa: E731
    out = [info["nullifier"] * bit(0)]
    f = info["fields"]
    if info.get("td1"):
        out += [f[k] * bit(k + 1) for k in range(6)]
        return out + [poseidon([f[6]]) * bit(7), poseidon([f[7]]) * bit(16), f[8] * bit(17)]
    for k, b in enumerate((1, 2, 3, 3, 4, 5, 6, 7)):
        out.append(f[k] * bit(b))
    return out


def batch_rows(batch, seed=0x9, distinct=64, depth=None, td1=False):
    """(batch, 842 | 858, 32) rows: `distinct` generated queries repeated (generation is host Python, ~40 ms each)."""
    rng = SplitMix64(seed)
    uniq = [pack(make_query(rng, depth=depth, td1=td1)[0]) for _ in range(min(batch, distinct))]
    out = np.empty((batch, uniq[0].shape[0], 32), dtype=np.uint8)
    for i in range(batch):
        out[i] = uniq[i % len(uniq)]
    return out
