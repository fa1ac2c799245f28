"""GPU parity for a mixed verification-flow batch: RSA-2048, RSA-4096
and ECDSA secp256r1 passports interleaved in one batch, grouped per instance by
pzkwit.mixed.MixedBatch; every witness equals the CPU oracle's and is returned in input order."""
import numpy as np
import pytest

from pzkwit import inputs as I, mixed

pytestmark = pytest.mark.gpu


def test_mixed_flows_match_oracle(oracle):
    flows = [dict(I.CANONICAL, sig=1), dict(I.CANONICAL, sig=2), dict(I.CANONICAL, sig=20)]
    gens = [I.PassportGen(seed=30 + k, n_keys=1, params=p, workers=1) for k, p in enumerate(flows)]
    order = [0, 2, 1, 0, 2]  # interleaved
    items = []
    for n, k in enumerate(order):
        items.append((flows[k], I.pack_register_inputs(gens[k].passport_at(n), flows[k])))
    wits, status = mixed.MixedBatch().run_host(items)
    assert (status == 0).all(), status
    for (prm, row), w in zip(items, wits):
        rc, ref = oracle.register_witness(oracle.register_params(**prm), row)
        assert rc == 0
        assert w.shape == ref.shape and np.array_equal(w, ref), prm["sig"]
