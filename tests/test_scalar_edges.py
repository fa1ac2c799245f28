"""CPU: edge scalars of the register path, pinned on the oracle by the constraint checker and independent math.

RegisterIdentity's key is BabyjubjubBase8Multiplication(skIdentity) over Num2Bits(254) + AliasCheck of sk
(identity.circom:112-120, babyjubjub/curve.circom:143-171, bitify/aliascheck.circom:7-14, compconstant.circom:7-55),
and the SMT key is Num2Bits(254) + AliasCheck of the pubkey hash (SMTVerifier.circom:109-176). getFakeIdenData's
sk has 62 hex digits (< 2^248), so the synthetic stream never sets bits 248-253 of either; a wallet's identity key
does. Here: sk in {0, 1, 2, 2^248, 2^251 + x, 2^253 + x, p - 2, p - 1}, and a passport whose pubkey hash is >= 2^253.
tests/test_gpu_scalar_edges.py runs the same rows through the device (both BabyJubJub cores)."""
import numpy as np
import pytest

from pzkwit import field, inputs as I

pyr1cs = pytest.importorskip("pyr1cs")

P = field.P
X = 0x1D2C3B4A5968778695A4B3C2D1E0F00112233445566778899AABBCCDDEEFF0
EDGE_SK = [0, 1, 2, 1 << 248, (1 << 251) + X % (1 << 200), (1 << 253) + X % (1 << 250), P - 2, P - 1]
SMT_OWN = 14  # layout.hpp RK_SMT_OWN: isVerified | root, leaf, key, siblings[80] | value


def edge_rows(gen, params=I.CANONICAL):
    rows = []
    for k, sk in enumerate(EDGE_SK):
        pp = dict(gen.passport_at(k))
        pp["sk"] = sk
        rows.append(I.pack_register_inputs(pp, params))
    return np.stack(rows)


def high_key_passport(gen, start=0):
    """a passport of the stream whose SMT key (the pubkey hash) has bit 253 set"""
    for i in range(start, start + 256):
        pp = gen.passport_at(i)
        if pp["pk_hash"] >> 253:
            return i, pp
    raise AssertionError("no pubkey hash >= 2^253 among 256 passports")


@pytest.fixture(scope="module")
def gen():
    return I.PassportGen(seed=0x5C, n_keys=8, workers=1)


def test_edge_scalars_oracle_satisfies_constraints(oracle, gen):
    from refmath import bjj_mul
    from test_r1cs import _ok, expected_uncovered
    prm = oracle.register_params(**I.CANONICAL)
    rows = edge_rows(gen)
    for sk, row in zip(EDGE_SK, rows):
        rc, w = oracle.register_witness(prm, row)
        assert rc == 0, (hex(sk), rc)
        _ok(pyr1cs.check_register(w, **I.CANONICAL), expected_uncovered(1))
        pk = int.from_bytes(w[4].tobytes(), "little")  # pkIdentityHash = Poseidon2(sk * Base8)
        if sk:
            x, y = bjj_mul(sk)
            assert pk == field.poseidon([x, y]), hex(sk)


def test_high_smt_key_oracle_satisfies_constraints(oracle, gen):
    from test_r1cs import _ok, expected_uncovered
    i, pp = high_key_passport(gen)
    prm = oracle.register_params(**I.CANONICAL)
    for depth in (0, 5):
        q = gen.passport_at(i, smt_depth=depth, smt_root=True)
        rc, w = oracle.register_witness(prm, I.pack_register_inputs(q))
        assert rc == 0
        _ok(pyr1cs.check_register(w, **I.CANONICAL), expected_uncovered(1))


def test_config4_root_verifies_on_oracle(oracle):
    """config 4's slaveMerkleRoot is the proof's root, computed by Python Poseidon over the
    SMTVerifier recurrence: the oracle's SMTVerifier must then set isVerified = 1 (passportVerificationBuilder.circom
    leaves it unenforced, so this is the only place the chain's root is compared with independent math)"""
    from test_gpu_register import region_table
    g = I.PassportGen(seed=4, n_keys=2, workers=1)
    off = [o for o, _, k in region_table(I.CANONICAL) if k == SMT_OWN][0]
    prm = oracle.register_params(**I.CANONICAL)
    for i, depth in enumerate((1, 2, 17, 40, 79)):
        pp = g.passport_at(i, smt_depth=depth, smt_root=True)
        rc, w = oracle.register_witness(prm, I.pack_register_inputs(pp))
        assert rc == 0
        assert int.from_bytes(w[off].tobytes(), "little") == 1, depth
        assert int.from_bytes(w[off + 1].tobytes(), "little") == pp["root"]
