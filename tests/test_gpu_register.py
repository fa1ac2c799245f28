"""GPU parity for RegisterIdentityBuilder(1,256,3,4,600,248,1,1496,3,256) (SURVEY.md §8d
configs 3 and 4): every witness element equals the CPU oracle's, the public outputs equal
independently computed values, and lane status is OK."""
import ctypes
import hashlib

import numpy as np
import pytest

from pzkwit import field, inputs as I, native

pytestmark = pytest.mark.gpu

KIND_NAMES = {0: "ONE", 1: "INCOPY", 2: "SHA_OWN", 3: "SHA_BLOCK", 4: "POSEIDON", 5: "MODMUL", 6: "VALUE",
              7: "BITS2NUM", 8: "NUM2BITS", 9: "DIGEST", 10: "TEMPMOD", 11: "FLOW", 12: "HCHUNK", 13: "RSA_OUT",
              14: "SMT_OWN", 15: "SMTHASH", 16: "LEVINS", 17: "SM", 18: "SMT_LEVEL", 19: "SWITCHER",
              20: "ISEQ_ROOT", 21: "BJJ_OWN", 22: "BJJ_STEPS"}


def region_table(params):
    L = native.lib()
    p = native.PzkParams(circuit=0)
    for k, v in native.param_fields(params).items():
        setattr(p, k, v)
    info = native.PzkInfo()
    n = ctypes.c_uint32()
    L.pzk_layout_query(ctypes.byref(p), ctypes.byref(info), ctypes.byref(n))
    out = []
    for i in range(n.value):
        off, ln, kd = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
        L.pzk_layout_region(ctypes.byref(p), i, ctypes.byref(off), ctypes.byref(ln), ctypes.byref(kd))
        out.append((off.value, ln.value, kd.value))
    return out


def mismatch_report(ref, got, regions, limit=12):
    bad = np.nonzero((ref != got).any(axis=1))[0]
    if bad.size == 0:
        return ""
    lines = ["%d mismatching elements" % bad.size]
    seen = {}
    for idx in bad:
        for ri, (off, ln, kd) in enumerate(regions):
            if off <= idx < off + ln:
                seen.setdefault(ri, []).append(int(idx - off))
                break
    for ri, locs in list(seen.items())[:limit]:
        off, ln, kd = regions[ri]
        e = off + locs[0]
        lines.append("region %d %s off=%d len=%d: %d bad, first local %s ref=%s got=%s" % (
            ri, KIND_NAMES.get(kd, kd), off, ln, len(locs), locs[:6],
            int.from_bytes(ref[e].tobytes(), "little"), int.from_bytes(got[e].tobytes(), "little")))
    return "\n".join(lines)


@pytest.fixture(scope="module")
def gen():
    return I.PassportGen(seed=3, n_keys=4)


def _check(oracle, params, batch_inputs):
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
    wit, st = inst.witness_batch_host(batch_inputs)
    prm = oracle.register_params(**params)
    regions = region_table(params)
    reports = []
    for b in range(batch_inputs.shape[0]):
        rc, ref = oracle.register_witness(prm, batch_inputs[b])
        assert rc == 0, "oracle check failed (site %d) on row %d" % (rc, b)
        rep = mismatch_report(ref, wit[b], regions)
        if rep:
            reports.append("row %d: %s" % (b, rep))
    assert not reports, "\n".join(reports)
    assert (st == 0).all(), st
    return wit


def test_register_canonical_matches_oracle(oracle, gen):
    rows = np.stack([I.pack_register_inputs(gen.passport_at(i)) for i in range(6)])
    wit = _check(oracle, I.CANONICAL, rows)
    # public outputs vs independent computation (process_passport.js / identity formulas)
    pp = gen.passport_at(0)
    sah = hashlib.sha256(pp["sa"]).digest()
    hb = [(sah[i // 8] >> (7 - i % 8)) & 1 for i in range(256)]
    n252 = sum(hb[i] << i for i in range(252))
    assert int.from_bytes(wit[0, 2].tobytes(), "little") == field.poseidon([n252])
    assert int.from_bytes(wit[0, 5].tobytes(), "little") == pp["root"]
    # pkIdentityHash = Poseidon2(sk * Base8) (identity.circom:112-120), dg1Commitment (identity.circom:89-109)
    from refmath import bjj_mul, dg1_commitment
    x, y = bjj_mul(pp["sk"])
    assert int.from_bytes(wit[0, 4].tobytes(), "little") == field.poseidon([x, y])
    assert int.from_bytes(wit[0, 3].tobytes(), "little") == dg1_commitment(pp["dg1"], pp["sk"])


def test_register_smt_depth_matches_oracle(oracle, gen):
    """config 4 shape: siblings non-zero up to a random depth (sequential SMT chain on GPU)."""
    rows = []
    for i, depth in enumerate([1, 7, 40, 79]):
        pp = gen.passport_at(100 + i, smt_depth=depth)
        pp["root"] = field.SplitMix64(i).fr()
        rows.append(I.pack_register_inputs(pp))
    _check(oracle, I.CANONICAL, np.stack(rows))


PARAM_VARIANTS = [
    dict(I.CANONICAL, doc=1),                      # TD1 chunking (190-bit dg1 chunks)
    dict(I.CANONICAL, aa=0),                       # no active authentication
    dict(I.CANONICAL, ec_blocks=5, ec_shift=640),  # longer encapsulated content
]


@pytest.mark.parametrize("params", PARAM_VARIANTS, ids=["td1", "aa0", "ec5"])
def test_register_param_variants_match_oracle(oracle, params):
    g = I.PassportGen(seed=11, n_keys=2, params=params)
    rows = np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=3 * i), params) for i in range(3)])
    _check(oracle, params, rows)


def test_register_rsa4096_matches_oracle(oracle):
    """SIGNATURE_TYPE 2: RSA-4096, 64-limb BigMultModP (k_rsa_core<64>, k_emit_mm<64>)."""
    params = dict(I.CANONICAL, sig=2)
    g = I.PassportGen(seed=12, n_keys=1, key_bits=4096, params=params)
    rows = np.stack([I.pack_register_inputs(g.passport_at(i), params) for i in range(2)])
    _check(oracle, params, rows)


def test_register_failing_checks_flag_lanes(oracle, gen):
    """Lanes that violate a constraint get the check-site code of the oracle (single failures) and
    do not disturb their neighbours; a multiply-failing lane reports a nonzero code."""
    pps = [gen.passport_at(200 + i) for i in range(4)]
    rows = np.stack([I.pack_register_inputs(p) for p in pps])
    ecL = I.CANONICAL["ec_blocks"] * 512
    rows[1, 1 + ecL + 10] ^= 1                         # one dg1 bit: dg1 hash != EC field -> flow (7)
    rows[2, rows.shape[1] - 2] = 0                     # siblings[79] != 0 -> SMTVerifier.circom:54 (13)
    rows[2, rows.shape[1] - 2, 0] = 5
    sig0 = 1 + ecL + 1024 + I.CANONICAL["dg15_blocks"] * 512 + 1024
    rows[3, sig0, 0] ^= 1                              # signature limb: EM checks fail (rsa.circom)
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL)
    _, st = inst.witness_batch_host(rows)
    prm = oracle.register_params(**I.CANONICAL)
    codes = [oracle.register_witness(prm, rows[b])[0] for b in range(4)]
    assert st[0] == 0 and codes[0] == 0
    assert st[1] == codes[1] == 7
    assert st[2] == codes[2] == 13
    assert codes[3] in (8, 9, 10) and st[3] in (8, 9, 10)


def test_register_rsa_outside_barrett_domain_matches_oracle(oracle, gen):
    """The cooperative RSA core (rsa_coop.hpp) uses Barrett reduction only when x*y < b^(2k), k the
    modulus' significant limbs, and exact Knuth D otherwise. A 31-limb modulus (top limb zero) with a
    full-width signature takes the Knuth D path for multiplications 0 and 16 and Barrett for the
    rest; every witness element must still equal the oracle's (which fails the EM checks)."""
    pps = [gen.passport_at(300 + i) for i in range(3)]
    rows = np.stack([I.pack_register_inputs(p) for p in pps])
    K = 32
    ecL = I.CANONICAL["ec_blocks"] * 512
    sig0 = 1 + ecL + 1024 + I.CANONICAL["dg15_blocks"] * 512 + 1024
    pk0 = sig0 + K
    for b in (1, 2):
        n = rows[b, pk0:pk0 + K].copy()
        rows[b, pk0:pk0 + K - 1] = n[1:]   # n' = n >> 64: 31 significant limbs, top limb >= 2^63
        rows[b, pk0 + K - 1] = 0
        rows[b, sig0 + K - 1] = 0
        rows[b, sig0 + K - 1, 0] = 0x39 * b  # x = sig: x^2 >= b^62 = b^(2k) -> outside Barrett's domain
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL)
    wit, st = inst.witness_batch_host(rows)
    prm = oracle.register_params(**I.CANONICAL)
    regions = region_table(I.CANONICAL)
    for b in range(3):
        rc, ref = oracle.register_witness(prm, rows[b])
        assert (rc == 0) == (b == 0) and (st[b] == 0) == (b == 0), (b, rc, st[b])
        rep = mismatch_report(ref, wit[b], regions)
        assert not rep, "row %d: %s" % (b, rep)


@pytest.mark.parametrize("params", [dict(I.CANONICAL, sig=3, dg_hash=160), dict(I.CANONICAL, sig=1, dg_hash=160, aa=0),
                                    dict(I.CANONICAL, sig=4, dg_hash=160), dict(I.CANONICAL, dg_hash=224)],
                         ids=["sig3-dg160", "sig1-dg160-aa0", "sig4-dg160", "sig1-dg224"])
def test_register_sha1_instances_match_oracle(oracle, params):
    """SHA-1 hashers inside RegisterIdentityBuilder (ShaHashChunks(B, 160) around Sha1HashChunks) for the DG
    hashes and, with SIGNATURE_TYPE 3, the EC / SA hashes and the PKCS#1 v1.5 SHA-1 check; a bad signature
    carries the rsa.circom hash-check code."""
    from test_gpu_ecdsa import _run
    g = I.PassportGen(seed=19, n_keys=2, params=params, workers=1)
    pps = [g.passport_at(0), g.passport_at(1, smt_depth=4), dict(g.passport_at(2))]
    pps[2]["sig"] = pps[2]["sig"] + 1
    rows = np.stack([I.pack_register_inputs(pp, params) for pp in pps])
    _, st, codes = _run(oracle, params, rows, expect_ok=False)
    assert codes == [0, 0, 8]
    assert list(st) == [0, 0, 8]
