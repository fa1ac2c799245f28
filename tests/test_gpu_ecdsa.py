"""GPU parity for RegisterIdentityBuilder with SIGNATURE_TYPE 20 (ECDSA secp256r1 + SHA-256,
SURVEY.md §8d config 5 and §8f rows f1/f2): every witness element of the 5.49 M-element O0
witness equals the CPU oracle's (oracle/ecdsa.inc.c), the lane status is OK, the public
outputs equal independent computations, and lanes whose signature does not verify carry the
check-site code of ecdsa.circom:81-83."""
import numpy as np
import pytest

from pzkwit import field, inputs as I, native
from test_gpu_register import KIND_NAMES, mismatch_report, region_table

pytestmark = pytest.mark.gpu

ECDSA = dict(I.CANONICAL, sig=20)
KIND_NAMES.update({24: "ECT", 25: "EC_U64", 26: "EC_CONST", 27: "EC_GM_RCC", 28: "EC_GM_EQ", 29: "EC_GM_SUM",
                   30: "EC_GM_STEP", 31: "EC_N2B", 32: "EC_B2N8", 33: "EC_SBITS", 34: "EC_SM_W0", 35: "EC_SM_DSW",
                   36: "EC_SM_SEL", 37: "EC_SM_RSW", 38: "EC_PKBITS", 39: "EC_B2N248"})


@pytest.fixture(scope="module")
def ec_gen():
    return I.PassportGen(seed=5, n_keys=2, params=ECDSA, workers=1)


def _run(oracle, params, rows, expect_ok=True):
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
    wit, st = inst.witness_batch_host(rows)
    prm = oracle.register_params(**params)
    regions = region_table(params)
    reports, codes = [], []
    for b in range(rows.shape[0]):
        rc, ref = oracle.register_witness(prm, rows[b])
        codes.append(rc)
        if rc == 0:
            rep = mismatch_report(ref, wit[b], regions)
            if rep:
                reports.append("row %d: %s" % (b, rep))
    assert not reports, "\n".join(reports)
    if expect_ok:
        assert codes == [0] * rows.shape[0]
        assert (st == 0).all(), st
    return wit, st, codes


def test_ecdsa_matches_oracle(oracle, ec_gen):
    pps = [ec_gen.passport_at(0), ec_gen.passport_at(1), ec_gen.passport_at(2, smt_depth=9)]
    pps[2]["root"] = field.SplitMix64(9).fr()
    rows = np.stack([I.pack_register_inputs(pp, ECDSA) for pp in pps])
    wit, _, _ = _run(oracle, ECDSA, rows)
    pp = pps[0]
    assert int.from_bytes(wit[0, 5].tobytes(), "little") == pp["root"] == field.poseidon([pp["pk_hash"]] * 2 + [1])


def test_ecdsa_td1_no_aa_matches_oracle(oracle):
    params = dict(ECDSA, doc=1, aa=0)
    g = I.PassportGen(seed=6, n_keys=1, params=params, workers=1)
    rows = np.stack([I.pack_register_inputs(g.passport_at(i), params) for i in range(2)])
    _run(oracle, params, rows)


def test_ecdsa_bad_signature_flags_lane(oracle, ec_gen):
    good = ec_gen.passport_at(3)
    bad = dict(ec_gen.passport_at(4))
    r, s = bad["sig"]
    bad["sig"] = (r, (s + 1) % I.P256_N)
    rows = np.stack([I.pack_register_inputs(good, ECDSA), I.pack_register_inputs(bad, ECDSA)])
    _, st, codes = _run(oracle, ECDSA, rows, expect_ok=False)
    assert codes == [0, 16]
    assert st[0] == 0 and st[1] == 16  # ecdsa.circom:81-83


def test_brainpool_matches_oracle(oracle):
    """SIGNATURE_TYPE 21 (brainpoolP256r1, general-a Jacobian doubling, its own fixed-base table):
    every element bit-exact; a tampered signature flags ecdsa.circom:81-83."""
    params = dict(I.CANONICAL, sig=21)
    g = I.PassportGen(seed=17, n_keys=2, params=params, workers=1)
    pps = [g.passport_at(0), g.passport_at(1, smt_depth=3), dict(g.passport_at(2))]
    r, s = pps[2]["sig"]
    pps[2]["sig"] = (r, (s + 1) % I.BP256.n)
    rows = np.stack([I.pack_register_inputs(pp, params) for pp in pps])
    _, st, codes = _run(oracle, params, rows, expect_ok=False)
    assert codes == [0, 0, 16]
    assert list(st) == [0, 0, 16]


@pytest.mark.parametrize("sig", [24, 25])
def test_p224_bp384_match_oracle(oracle, sig):
    """SIGNATURE_TYPE 24 (secp224r1: 7 x 32-bit chunks, a = -3 doubling, SHA-224 signed attributes over a SHA-256
    encapsulated-content hash) and 25 (brainpoolP384r1: 6 x 64-bit chunks, 12-word Montgomery fields, SHA-384 in
    1024-bit blocks): every element of the 5.66 M / 10.9 M-element witness bit-exact against the generic CPU
    restatement (oracle/ecdsa.inc.c, itself checked constraint by constraint by oracle/r1cs_check.c); a tampered s
    flags ecdsa.circom:81-83."""
    params = I.instance_params(sig)
    g = I.PassportGen(seed=23 + sig, n_keys=2, params=params, workers=1)
    pps = [g.passport_at(0), g.passport_at(1, smt_depth=4), dict(g.passport_at(2))]
    pps[1]["root"] = field.SplitMix64(4).fr()
    r, s = pps[2]["sig"]
    pps[2]["sig"] = (r, (s + 1) % I.EC_CURVES[sig].n)
    rows = np.stack([I.pack_register_inputs(pp, params) for pp in pps])
    wit, st, codes = _run(oracle, params, rows, expect_ok=False)
    assert codes == [0, 0, 16]
    assert list(st) == [0, 0, 16]
    pp = pps[0]
    assert int.from_bytes(wit[0, 5].tobytes(), "little") == pp["root"] == field.poseidon([pp["pk_hash"]] * 2 + [1])
