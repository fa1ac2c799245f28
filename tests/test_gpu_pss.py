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

KIND_NAMES.update({40: "PSS_OWN", 41: "PSS_B2N8", 42: "PSS_MGF", 43: "PSS_CTR", 44: "PSS_XOR", 47: "SHA5_OWN", 48: "SHA5_BLOCK"})


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


@pytest.mark.parametrize("variant", ["dg384", "dg256-noaa", "ec-aa"])
def test_pss384_sig13_matches_oracle(oracle, variant):
    """SIGNATURE_TYPE 13: RSA-2048 PSS over SHA-384 (salt 48, Mgf1Sha384 with 5 SHA-384 blocks, one-block
    SHA-384 M' hasher; rsaPss.circom:18-254, mgf1.circom:5-68) with SHA-384 EC / SA hashers in 1024-bit
    blocks (k_sha_core algo 3, k_emit_sha512 with the ShaHashChunks wrapper; the derived-message hashers
    through E_SHA5D). DG hash 384, or SHA-256 DG hashes without DG15; every element vs the oracle, plus a
    failing lane per PSS check site."""
    params = I.instance_params(13)
    if variant == "dg256-noaa":
        params = dict(params, dg_hash=256, aa=0, dg15_blocks=0)
    elif variant == "ec-aa":
        params = dict(params, aa=20)
    g = I.PassportGen(seed=31, n_keys=2, params=params, workers=1)
    pps = [g.passport_at(0), g.passport_at(1, smt_depth=4)]
    pps[1]["root"] = 4242
    if variant == "dg384":
        bad = dict(g.passport_at(2))
        bad["sig"] += 1
        other = dict(g.passport_at(3))
        import hashlib
        other["sig"] = I.pss_sign(g.keys[1], other["sa"] + b"x", bytes(48), hashlib.sha384)
        pps += [bad, other]
        _, st, codes = _run(oracle, params, np.stack([I.pack_register_inputs(pp, params) for pp in pps]),
                            expect_ok=False)
        assert codes == [0, 0, 17, 18] and list(st) == codes  # rsaPss.circom:73, :225
    else:
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
