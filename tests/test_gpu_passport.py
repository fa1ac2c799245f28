"""GPU: EF.SOD files -> bulk preprocessor (pzk_passport_inputs) -> pzk_witness_batch, end to end.
Synthetic passports with real SOD DER (pzkwit.sodgen) for SIG 1 (canonical LDS layout), PSS and ECDSA
signers; every lane verifies (status OK) and sampled rows equal the CPU oracle element for element."""
import numpy as np
import pytest

from pzkwit import inputs as I, native, passport as PP, sodgen
from test_gpu_register import _check

pytestmark = pytest.mark.gpu


def _batch(sig, n, **opt):
    key = sodgen.signer_key(sig)
    pps = [sodgen.make_passport(sig, key, i, **opt) for i in range(n)]
    if isinstance(key, I.EcKey):
        pkh = I.ecdsa_pk_hash(key.q, key.curve.p.bit_length())
    else:
        a = I.chunk_limbs(key.n, 64, 15)
        pkh = I.poseidon([(a[3 * i] << 128) + (a[3 * i + 1] << 64) + a[3 * i + 2] for i in range(5)])
    ident = []
    for pp in pps:
        sk_hex, root_hex, _ = I.fake_iden_data(pp["ec"], pkh)  # getFakeIdenData (process_passport.js:628-657)
        ident.append(PP.identity_elements(int(root_hex, 16), int(sk_hex, 16)))
    return pps, np.stack(ident)


@pytest.mark.parametrize("sig,opt", [(1, {}), (11, {}), (20, {}), (25, {"signing_time": False}), (1, {"dg15": False, "n_dgs": 3})],
                         ids=["sig1", "sig11", "sig20", "sig25", "sig1_noaa"])
def test_sod_to_witness(oracle, sig, opt):
    pps, ident = _batch(sig, 24, **opt)
    params = PP.parse(pps[0])["params"]
    assert params["sig"] == sig
    rows, st = PP.input_rows(params, pps, ident)
    assert (st == 0).all(), st
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
    _, wst = inst.witness_batch_host(rows)
    assert (wst == 0).all(), wst
    _check(oracle, params, rows[[0, 23]])
