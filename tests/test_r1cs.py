"""CPU: the constraint checker (oracle/r1cs_check.c) over oracle witnesses.

The reference accepts a witness when every constraint of the compiled circuit holds
(circom_tester checkConstraints, test/automatisationTest.js:51). r1cs_check.c restates the
constraints of every template on the path from the .circom sources — walking the component tree
itself in the --O0 numbering — and evaluates them on a witness. Here it pins the oracle's
intermediate signals (values the witness restatement computes but no reference-run fixture covers):
a witness passes only if the checker's own allocation matches the oracle's signal for signal and
every `<==` / `===` holds. tests/test_gpu_r1cs.py applies the same checker to device witnesses.

Signals no constraint reads: the declared-but-never-assigned tmpResult entries of
BigMultNonEqualOverflow (bigIntHelpers.circom:83-118, the triangle outside each row's sum), 992 per
BigMultModP(64,32,32,32) and 4,032 per BigMultModP(64,64,64,64); they must hold 0.
"""
import numpy as np
import pytest

from pzkwit import field, inputs as I

pyr1cs = pytest.importorskip("pyr1cs")

UNASSIGNED_PER_BMM = {32: 992, 64: 4032, 48: 4512}
# BigMultModP instances per PowerMod (exp_to_bits, bigIntFunc.circom:590-616): 65537 -> 16 squarings + 1,
# 3 -> 1 + 1, 37187 -> 15 + 5; SIG 3 / 4 add the two never-assigned hashed_chunks of rsa.circom:81
N_BMM = {1: 17, 2: 17, 3: 17, 4: 20, 10: 2, 11: 17, 12: 17, 13: 17, 14: 17}
EXTRA = {3: 2, 4: 2}
# ECDSA (verifyECDSABits over N chunks): every BigMultNonEqualOverflow(G, N) leaves N (N - 1) tmpResult entries
# unassigned, per EllipticCurveDouble 9 products, per EllipticCurveAdd 8, per BigMultModP 2 (PointOnCurve 5,
# PointOnTangent 4, PointOnLine 3); P-256: 260 doubles (precompute 7, scalar mult 4 x 63, second dummy 1) and 102 adds
# (precompute 7, scalar mult 63, generator mult 31, final 1) and 4 BigMultModP; plus EllipicCurveScalarGeneratorMult's
# never-assigned resultingPointsLeft/Left2/Right/Right2 (4 x PARTS x 2N) and resultingPoints[PARTS - 1] (2N)
# (ec/curve.circom:812-816, 904)
def ecdsa_uncovered(sig):
    n, cs = I.EC_CHUNKS[sig]
    wins, parts = n * cs // 4, n * cs // 8
    dbl, add = 8 + 4 * (wins - 1), 7 + (wins - 1) + (parts - 1) + 1
    return n * (n - 1) * (9 * dbl + 8 * add + 4 * 2) + 4 * parts * 2 * n + 2 * n


ECDSA_UNCOVERED = ecdsa_uncovered(20)
assert ECDSA_UNCOVERED == 12 * (260 * 9 + 102 * 8 + 4 * 2) + 4 * 32 * 8 + 8


def expected_uncovered(sig):
    if sig >= 20:
        return ecdsa_uncovered(sig)
    return N_BMM[sig] * UNASSIGNED_PER_BMM[I.sig_input_len(sig)] + EXTRA.get(sig, 0)


def _ok(res, uncovered):
    rc, r = res
    assert r["oob"] == 0 and r["n_failed"] == 0, r
    assert r["n_uncovered"] == uncovered and r["n_uncovered_nonzero"] == 0, r
    assert rc == 0, r
    return r


def test_poseidon_circuits(oracle):
    for n in (1, 2, 3, 4, 5):
        for ins in ([0] * n, [field.P - 1 - i for i in range(n)], [field.SplitMix64(n).fr() for _ in range(n)]):
            rc, w = oracle.poseidon_witness(ins)
            assert rc == 0
            _ok(pyr1cs.check_poseidon(w, n), 0)


def test_sha1_circuit(oracle):
    for blocks in (1, 3):
        m = bytes(range(64 * blocks - 9))
        r = np.zeros((512 * blocks, 32), np.uint8)
        r[:, 0] = I.bits_msb_first(I.sha_pad(m))
        rc, w = oracle.sha1_witness(r, blocks)
        assert rc == 0
        _ok(pyr1cs.check_sha1(w, blocks), 0)


@pytest.mark.parametrize("out_bits", [384, 512])
def test_sha512_circuits(oracle, out_bits):
    """Sha384HashChunks / Sha512HashChunks (sha2/sha384, sha512/*.circom): every constraint of the schedule,
    the 80 compression rounds (64-bit GetLastNBits decompositions of sums up to 67 bits) and the chunk
    wiring holds on oracle witnesses; one flipped round bit breaks one."""
    rng = np.random.default_rng(out_bits)
    for blocks in (1, 2):
        m = rng.integers(0, 256, 128 * blocks - 40, dtype=np.uint8).tobytes()
        r = np.zeros((1024 * blocks, 32), np.uint8)
        r[:, 0] = I.bits_msb_first(I.sha_pad(m, 1024))
        rc, w = oracle.sha512_witness(r, blocks, out_bits)
        assert rc == 0
        _ok(pyr1cs.check_sha512(w, blocks, out_bits), 0)
    w = w.copy()
    k = 1 + out_bits + 2048 + 512 * 3 + 512 + 94480 + 5000  # inside block 0's rounds
    w[k, 0] ^= 1
    rc, rep = pyr1cs.check_sha512(w, blocks, out_bits)
    assert rc != 0 and rep["n_failed"] > 0


def test_sha256_config2(oracle):
    _, rows = I.sha256_config2_batch(3, seed=2, blocks=6)
    for r in rows:
        rc, w = oracle.sha256_witness(r, 6)
        assert rc == 0
        rep = _ok(pyr1cs.check_sha256(w, 6), 0)
        assert rep["size_walked"] == w.shape[0]


REGISTER_CASES = [
    ("canonical", dict(I.CANONICAL), 0),
    ("canonical_smt7", dict(I.CANONICAL), 7),
    ("canonical_smt79", dict(I.CANONICAL), 79),
    ("rsa4096", dict(I.CANONICAL, sig=2), 3),
    ("td1_no_aa", dict(I.CANONICAL, doc=1, aa=0), 0),
    ("ec_aa", dict(I.CANONICAL, aa=20), 0),
    ("dg224", dict(I.CANONICAL, dg_hash=224, dg15_shift=1496), 0),
    ("sig3_sha1", I.instance_params(3), 2),
    ("sig4_rsa3072_sha1", I.instance_params(4), 0),
    ("sig10_pss_e3", I.instance_params(10), 4),
    ("sig11_pss", I.instance_params(11), 0),
    ("sig12_pss_salt64", I.instance_params(12), 0),
    ("sig13_pss_sha384", I.instance_params(13), 0),
    ("sig13_dg256_no_dg15", dict(I.instance_params(13), dg_hash=256, aa=0, dg15_blocks=0), 2),
    ("sig14_pss3072", I.instance_params(14), 1),
    ("sig20_ecdsa_p256", I.instance_params(20), 0),
    ("sig21_ecdsa_brainpool", I.instance_params(21), 3),
    ("sig24_ecdsa_p224", I.instance_params(24), 2),
    ("sig24_dg256", dict(I.instance_params(24), dg_hash=256), 0),
    ("sig25_ecdsa_brainpool384", I.instance_params(25), 0),
]


def _register_witness(oracle, params, depth, idx=0, seed=0x31):
    g = I.PassportGen(seed=seed, n_keys=2, params=params, workers=1)
    pp = g.passport_at(idx, smt_depth=depth)
    if pp["root"] is None:
        pp["root"] = field.SplitMix64(idx).fr()  # the SMT check is not enforced (passportVerificationBuilder.circom:240)
    row = I.pack_register_inputs(pp, params)
    rc, w = oracle.register_witness(oracle.register_params(**params), row)
    return rc, w


@pytest.mark.parametrize("name,params,depth", REGISTER_CASES, ids=[c[0] for c in REGISTER_CASES])
def test_register_oracle_witness_satisfies_constraints(oracle, name, params, depth):
    rc, w = _register_witness(oracle, params, depth)
    assert rc == 0
    r = _ok(pyr1cs.check_register(w, **params), expected_uncovered(params["sig"]))
    assert r["size_walked"] == w.shape[0]


def test_tampered_signals_break_constraints(oracle):
    """One flipped bit anywhere (a SHA round bit, a Karatsuba node, a BigIntIsZero carry, a Poseidon
    S-box, a BabyJubJub ladder point, ...) violates at least one constraint."""
    rc, w = _register_witness(oracle, dict(I.CANONICAL), 3)
    assert rc == 0
    rng = np.random.default_rng(7)
    covered = pyr1cs.check_register(w, **I.CANONICAL)[1]
    assert covered["n_failed"] == 0
    for idx in list(rng.integers(1, w.shape[0], 40)) + [2, 5, w.shape[0] - 1]:
        v = w.copy()
        v[idx, 0] ^= 1
        if int.from_bytes(v[idx].tobytes(), "little") >= field.P:
            continue
        rc, r = pyr1cs.check_register(v, **I.CANONICAL)
        assert rc != 0 and (r["n_failed"] > 0 or r["n_uncovered_nonzero"] > 0), idx


def test_invalid_ecdsa_signature_fails_constraints(oracle):
    """A tampered ECDSA s: the oracle flags its site and the witness violates the constraints of
    verifyECDSABits (ecdsa.circom:88-90 x1 mod n === r, or an EC point check)."""
    params = I.instance_params(20)
    g = I.PassportGen(seed=0x33, n_keys=2, params=params, workers=1)
    pp = g.passport_at(0)
    r_, s_ = pp["sig"]
    pp["sig"] = (r_, s_ ^ 1)
    rc, w = oracle.register_witness(oracle.register_params(**params), I.pack_register_inputs(pp, params))
    assert rc != 0
    rc2, r = pyr1cs.check_register(w, **params)
    assert rc2 != 0 and r["n_failed"] > 0


def test_invalid_signature_witness_fails_constraints(oracle):
    """A passport whose signature does not verify: the oracle flags its check site, and the same
    witness violates the RSA constraints (rsa.circom:46-67)."""
    g = I.PassportGen(seed=0x32, n_keys=2, workers=1)
    pp = g.passport_at(1)
    pp["sig"] = (pp["sig"] + 1) % pp["n"]
    rc, w = oracle.register_witness(oracle.register_params(**I.CANONICAL), I.pack_register_inputs(pp))
    assert rc != 0
    rc2, r = pyr1cs.check_register(w, **I.CANONICAL)
    assert rc2 != 0 and r["n_failed"] > 0
    assert "RsaVerifyPkcs1v15" in r["first_template"] or "BigIntIsZero" in r["first_template"], r
