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


def test_mixed_batch_sharded_properties(oracle):
    """A 60-passport config-5 batch (40 % RSA-2048, 30 % RSA-4096, 30 % ECDSA P-256, shuffled) cut
    into two cost-balanced shards as bench.py --gpus 2 would, each shard run as one grouped batch:
    every lane's checks hold, each row has its own flow's witness size, witness[0] = 1 and
    passportHash (witness[2]) = Poseidon(SHA-256(SA) low 252 bits) for every row, and the first row of
    each flow in each shard plus the batch's last row are bit-exact against the CPU oracle."""
    import hashlib

    from pzkwit import field
    flows = [dict(I.CANONICAL, sig=1), dict(I.CANONICAL, sig=2), dict(I.CANONICAL, sig=20)]
    gens = [I.PassportGen(seed=50 + k, n_keys=2, params=p, workers=1) for k, p in enumerate(flows)]
    kinds = np.random.default_rng(5).permutation([0] * 24 + [1] * 18 + [2] * 18)
    pps = [gens[k].passport_at(n) for n, k in enumerate(kinds)]
    items = [(flows[k], I.pack_register_inputs(pp, flows[k])) for k, pp in zip(kinds, pps)]
    costs = [mixed.witness_cost(prm) for prm, _ in items]
    sizes = {k: mixed.witness_cost(flows[k]) // 32 for k in range(3)}
    shards = [mixed.shard_by_cost(costs, 2, r) for r in range(2)]
    assert shards[0][0] == 0 and shards[0][1] == shards[1][0] and shards[1][1] == len(items)
    mb = mixed.MixedBatch()
    for lo, hi in shards:
        wits, status = mb.run_host(items[lo:hi])
        assert (status == 0).all(), status
        seen = set()
        for n, w in enumerate(wits, start=lo):
            k = int(kinds[n])
            assert w.shape == (sizes[k], 32)
            assert int.from_bytes(w[0].tobytes(), "little") == 1
            h = hashlib.sha256(pps[n]["sa"]).digest()
            bits = [(h[i // 8] >> (7 - i % 8)) & 1 for i in range(252)]
            assert int.from_bytes(w[2].tobytes(), "little") == field.poseidon([sum(b << i for i, b in enumerate(bits))]), n
            if k not in seen or n == len(items) - 1:
                seen.add(k)
                prm, row = items[n]
                rc, ref = oracle.register_witness(oracle.register_params(**prm), row)
                assert rc == 0 and np.array_equal(w, ref), (n, prm["sig"])
        del wits
