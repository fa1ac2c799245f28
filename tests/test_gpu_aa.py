"""GPU parity for the active-authentication variants of RegisterIdentityBuilder (SURVEY.md §8f row
f1): AA_SIGNATURE_ALGO 2 (RSA key; the DG15 IsEqual inputs of PassportVerificationFlow are scaled
by the raw value, passportVerificationFlow.circom:45-46,73-74, so their IsZero inverses are 1/±2)
and 20 / 23 (EC key hashed as Poseidon2 of its low bits, identity.circom:51-84). Every witness
element equals the CPU oracle's and lane status is OK."""
import numpy as np
import pytest

from pzkwit import inputs as I
from test_gpu_ecdsa import _run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("params", [dict(I.CANONICAL, aa=2), dict(I.CANONICAL, aa=20),
                                    dict(I.CANONICAL, sig=20, aa=23)], ids=["rsa-aa2", "ec-aa20", "ecdsa-ec-aa23"])
def test_aa_variants_match_oracle(oracle, params):
    g = I.PassportGen(seed=14, n_keys=1, params=params, workers=1)
    _run(oracle, params, np.stack([I.pack_register_inputs(g.passport_at(i), params) for i in range(2)]))
