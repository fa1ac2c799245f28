"""GPU: the register path at the scalar edges of tests/test_scalar_edges.py — skIdentity in {0, 1, 2, 2^248,
2^251 + x, 2^253 + x, p - 2, p - 1} and a pubkey hash >= 2^253 as the SMT key — element for element against the
oracle through both BabyJubJub cores (the scratch kernel k_bjj_core, the default, and k_bjj_core_rc, PZK_BJJ=rc),
and config 4's proofs (depths 1-79, slaveMerkleRoot = the proof's root): the device's SMT chain sets
isVerified = 1 on every lane (identity.circom:112-120, babyjubjub/curve.circom:143-171, aliascheck.circom:7-14,
SMTVerifier.circom:109-176)."""
import os

import numpy as np
import pytest

from pzkwit import inputs as I, native
from test_gpu_register import mismatch_report, region_table
from test_scalar_edges import EDGE_SK, SMT_OWN, edge_rows, high_key_passport

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gen():
    return I.PassportGen(seed=0x5C, n_keys=8, workers=1)


@pytest.mark.parametrize("core", ["rc", "scratch"])
def test_edge_scalars_match_oracle(oracle, gen, core):
    rows = edge_rows(gen)
    i, _ = high_key_passport(gen)
    rows = np.concatenate([rows, I.pack_register_inputs(gen.passport_at(i, smt_depth=6, smt_root=True))[None]])
    old = os.environ.get("PZK_BJJ")
    os.environ["PZK_BJJ"] = core  # read per call: set for the instance's whole life
    try:
        inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL)
        wit, st = inst.witness_batch_host(rows)
        del inst
    finally:
        if old is None:
            os.environ.pop("PZK_BJJ", None)
        else:
            os.environ["PZK_BJJ"] = old
    prm = oracle.register_params(**I.CANONICAL)
    regions = region_table(I.CANONICAL)
    for b in range(rows.shape[0]):
        rc, ref = oracle.register_witness(prm, rows[b])
        assert rc == 0 and st[b] == 0, (b, rc, st[b])
        rep = mismatch_report(ref, wit[b], regions)
        assert not rep, "row %d (sk %s): %s" % (b, hex(EDGE_SK[b]) if b < len(EDGE_SK) else "pk>=2^253", rep)


def test_config4_roots_verify_on_device(oracle):
    """128 config-4 passports (seed 0x4, depth uniform 1-79, root computed in Python): every lane's device
    isVerified = 1 and root = the input; three rows element for element against the oracle"""
    import bench
    rows = bench.make_register_inputs(128, 0, seed=4, sig=1, workers=4, smt_depth="1-79", smt_root=True)
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL)
    wit, st = inst.witness_batch_host(rows)
    assert (st == 0).all()
    off = [o for o, _, k in region_table(I.CANONICAL) if k == SMT_OWN][0]
    assert (wit[:, off, 0] == 1).all() and not wit[:, off, 1:].any()
    assert (wit[:, off + 1] == rows[:, 0]).all()  # root | slaveMerkleRoot (input 0)
    prm = oracle.register_params(**I.CANONICAL)
    regions = region_table(I.CANONICAL)
    for b in (0, 63, 127):
        rc, ref = oracle.register_witness(prm, rows[b])
        assert rc == 0
        rep = mismatch_report(ref, wit[b], regions)
        assert not rep, "row %d: %s" % (b, rep)
