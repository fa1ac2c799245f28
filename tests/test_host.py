"""CPU: host-side logic — input formats (process_passport.js), JSON marshalling with the
witness calculator's error semantics, sharding and the multi-process (gloo) result gather."""
import hashlib
import os

import numpy as np
import pytest

from pzkwit import dist as D, inputs as I, witness_calculator as WC
from pzkwit.field import P


def test_sha_pad_matches_fips_padding():
    for L in (0, 55, 56, 63, 64, 93, 165, 247):
        m = bytes(range(256))[:L] if L <= 256 else b"x" * L
        pad = I.sha_pad(m)
        assert len(pad) % 64 == 0
        assert pad[:L] == m and pad[L] == 0x80
        assert int.from_bytes(pad[-8:], "big") == 8 * L


def test_synthetic_passport_structure():
    g = I.PassportGen(seed=3, n_keys=2)
    pp = g.passport_at(7)
    assert len(pp["dg1"]) == 93 and len(I.sha_pad(pp["dg1"])) == 128
    assert len(I.sha_pad(pp["dg15"])) == 3 * 64
    assert len(I.sha_pad(pp["ec"])) == 4 * 64
    assert pp["ec"][31:63] == hashlib.sha256(pp["dg1"]).digest()
    assert pp["ec"][184] == 0x0F and pp["ec"][187:219] == hashlib.sha256(pp["dg15"]).digest()
    assert pp["sa"][75:107] == hashlib.sha256(pp["ec"]).digest()
    # deterministic per index
    assert g.passport_at(7)["sig"] == pp["sig"]
    # RSA PKCS#1 v1.5 verifies
    key = g.keys[7 % 2]
    em = pow(pp["sig"], key.e, key.n).to_bytes(256, "big")
    assert em.startswith(b"\x00\x01\xff") and em.endswith(hashlib.sha256(pp["sa"]).digest())


def test_json_marshalling_equals_packed_inputs():
    g = I.PassportGen(seed=3, n_keys=2)
    pp = g.passport_at(1)
    js = I.passport_json(pp)
    groups = [("slaveMerkleRoot", 0, 1), ("encapsulatedContent", 1, 2048), ("dg1", 2049, 1024),
              ("dg15", 3073, 1536), ("signedAttributes", 4609, 1024), ("signature", 5633, 32),
              ("pubkey", 5665, 32), ("slaveMerkleInclusionBranches", 5697, 80), ("skIdentity", 5777, 1)]
    buf = WC.marshal_inputs(groups, 5778, js)
    assert np.array_equal(buf, I.pack_register_inputs(pp))


def test_json_marshalling_errors():
    groups = [("a", 0, 2), ("b", 2, 1)]
    with pytest.raises(WC.WitnessError, match="Signal c not found"):
        WC.marshal_inputs(groups, 3, {"a": [1, 2], "c": 1})
    with pytest.raises(WC.WitnessError, match="Not enough values for input signal a"):
        WC.marshal_inputs(groups, 3, {"a": [1], "b": 1})
    with pytest.raises(WC.WitnessError, match="Too many values for input signal a"):
        WC.marshal_inputs(groups, 3, {"a": [1, 2, 3], "b": 1})
    with pytest.raises(WC.WitnessError, match="Not all inputs have been set"):
        WC.marshal_inputs(groups, 3, {"a": [1, 2]})
    buf = WC.marshal_inputs(groups, 3, {"a": [[-1], ["0x10"]], "b": str(P + 5)})
    assert int.from_bytes(buf[0].tobytes(), "little") == P - 1
    assert int.from_bytes(buf[1].tobytes(), "little") == 16
    assert int.from_bytes(buf[2].tobytes(), "little") == 5


def test_shard_range_partitions():
    for total in (1, 7, 4096, 32768):
        for world in (1, 2, 3, 8):
            spans = [D.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = D.shard_range(10, world, rank)
    st = torch.tensor([i % 3 == 0 for i in range(lo, hi)], dtype=torch.int32)
    pub = torch.zeros((hi - lo, 5, 32), dtype=torch.uint8)
    pub[:, 0, 0] = torch.arange(lo, hi, dtype=torch.uint8)
    s, p = D.gather_results(dist, st, pub)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
    if rank == 0:
        q.put((s.tolist(), p[:, 0, 0].tolist(), float(t.item())))
    dist.destroy_process_group()


def test_two_rank_gloo_gather():
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    st, ids, t = q.get(timeout=120)
    for p in ps:
        p.join(60)
    assert ids == list(range(10))
    assert st == [1 if i % 3 == 0 else 0 for i in range(10)]
    assert t == 2.0


def test_mixed_shard_by_cost_balances_bytes():
    """Config 5: a mixed RSA-2048 / RSA-4096 / ECDSA batch sharded by .wtns bytes:
    shards tile the batch in order and each is within one witness of the even byte split."""
    from pzkwit import mixed
    rng = np.random.default_rng(5)
    sigs = rng.choice([1, 2, 20], size=997, p=[0.4, 0.3, 0.3])
    costs = [mixed.witness_cost(dict(I.CANONICAL, sig=int(s))) for s in sigs]
    assert costs[list(sigs).index(20)] == 32 * 5488453
    for world in (1, 2, 8):
        bounds = [mixed.shard_by_cost(costs, world, r) for r in range(world)]
        assert bounds[0][0] == 0 and bounds[-1][1] == len(costs)
        assert all(bounds[r][1] == bounds[r + 1][0] for r in range(world - 1))
        share = sum(costs) / world
        for lo, hi in bounds:
            assert abs(sum(costs[lo:hi]) - share) <= max(costs)
