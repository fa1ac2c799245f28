"""GPU parity for RegisterIdentityBuilder with RSA-PSS signatures (SIGNATURE_TYPE 10, 11, 12:
RSA-2048, SHA-256, MGF1-SHA-256; e = 3 / 65537, salt 32 / 64 bytes; 14: RSA-3072, whose 48-limb
BigMultModP multiplies by schoolbook BigMultNonEqualOverflow):
every element of the O0 witness (3.29 M / 3.65 M elements) equals the CPU oracle's
(VerifyRsaPssSig restatement, oracle/witness_oracle.c), lane status is OK, and lanes whose
signature fails carry the check-site code of rsaPss.circom:73 / :182."""
import numpy as np
import pytest

from pzkwit import inputs as I
from test_gpu_ecdsa import _run
from test_gpu_register import KIND_NAMES

pytestmark = pytest.mark.gpu

KIND_NAMES.update({40: "PSS_OWN", 41: "PSS_B2N8", 42: "PSS_MGF", 43: "PSS_CTR", 44: "PSS_XOR"})


@pytest.fixture(scope="module")
def gens():
    return {sig: I.PassportGen(seed=12, n_keys=2, params=dict(I.CANONICAL, sig=sig), workers=1) for sig in (10, 11, 12, 14)}


@pytest.mark.parametrize("sig", [10, 11, 12, 14])
def test_pss_matches_oracle(oracle, gens, sig):
    params = dict(I.CANONICAL, sig=sig)
    g = gens[sig]
    pps = [g.passport_at(0), g.passport_at(1), g.passport_at(2, smt_depth=5)]
    pps[2]["root"] = 12345
    _run(oracle, params, np.stack([I.pack_register_inputs(pp, params) for pp in pps]))


def test_pss_td1_no_aa_matches_oracle(oracle):
    params = dict(I.CANONICAL, sig=12, doc=1, aa=0)
    g = I.PassportGen(seed=13, n_keys=1, params=params, workers=1)
    _run(oracle, params, np.stack([I.pack_register_inputs(g.passport_at(i), params) for i in range(2)]))


def test_pss_bad_signatures_flag_lanes(oracle, gens):
    params = dict(I.CANONICAL, sig=11)
    g = gens[11]
    good = g.passport_at(3)
    trailer = dict(g.passport_at(4))
    trailer["sig"] += 1
    other = dict(g.passport_at(5))
    other["sig"] = I.pss_sha256_sign(g.keys[5 % len(g.keys)], other["sa"] + b"x", bytes(32))
    rows = np.stack([I.pack_register_inputs(pp, params) for pp in (good, trailer, other)])
    _, st, codes = _run(oracle, params, rows, expect_ok=False)
    assert codes == [0, 17, 18]
    assert list(st) == [0, 17, 18]  # rsaPss.circom:73, :182
