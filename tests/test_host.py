"""CPU: host-side logic — input formats (process_passport.js), JSON marshalling with the
witness calculator's error semantics, sharding and the multi-process (gloo) result gather."""
import hashlib
import os
import sys

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


def test_mixed_bench_rows_are_the_flow_groups():
    """Config 5 in bench.py: rank 0 makes each shard's rows grouped per flow and padded to the widest
    flow's row; a rank cuts its flows' compact rows back out (bench_mixed). The grouped rows equal the
    flows' own packed inputs of the same global passports, and the shards tile the job."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from pzkwit import native
    sigs, flows, costs, shards = bench._mixed_plan(24, 2)
    assert shards[0][0] == 0 and shards[0][1] == shards[1][0] and shards[1][1] == 48
    n_in_max = max(native.layout_inputs(flows[sg]) for sg, _ in bench.MIX)
    lo, hi = shards[1]
    rows = bench._mixed_host_rows(sigs, lo, hi, n_in_max, 1)
    pos = 0
    for sg, idx in bench._mixed_groups(sigs, lo, hi).items():
        assert all(int(sigs[i]) == sg for i in idx) and idx == sorted(idx)
        n_keys = {1: 64, 2: 8, 20: 64}[sg]
        g = I.PassportGen.shared(5, n_keys, sg)
        for k in (0, len(idx) - 1):
            want = I.pack_register_inputs(g.passport_at(idx[k]), g.params)
            assert (rows[pos + k, : g.n_inputs] == want).all()
            assert not rows[pos + k, g.n_inputs:].any()
        pos += len(idx)
    assert pos == hi - lo


class _StubInst:
    """timing / phase_info of a libpzkwit instance, for bench.report without a GPU"""

    def timing(self, reset=False):
        return {"emit_sha": (2.0, 4)}

    def phase_info(self):
        return [("emit_sha", "k_emit_sha", 1000)]


class _StubEngine:
    """bench.GpuEngine's interface on the CPU: 'witness' = the row's first 4 input elements, status =
    bit 0 of the row (config-2 message bits), so the gather's order can be checked."""

    def __init__(self, args, workload, dev):
        import torch
        nin = {"query": 842, "register": 5778}.get(workload, 3072)
        self.torch, self.NIN, self.W, self.n_pub, self.inst = torch, nin, nin + 300, 4, _StubInst()
        self.layout = "stub"

    def setup(self, d_in, batch, sub, slots, steps):
        self.rows = d_in.view(batch, self.NIN, 32)
        self.d_st = self.torch.zeros((steps, batch), dtype=self.torch.int32)

    def step(self, k, timing):
        self.d_st[k] = self.rows[:, 0, 0].to(self.torch.int32)

    def sync(self):
        pass

    def statuses(self, steps):
        return self.d_st[:steps]

    def public_pass(self):
        return self.rows[:, 0, 0].to(self.torch.int32).clone(), self.rows[:, : self.n_pub].clone()


def _bench_rank(rank, world, port, q, workload="sha256"):
    import argparse
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = argparse.Namespace(workload=workload, batch=6, sub=None, slots=1, steps=2, warmup=1,
                              sig_eff=1 if workload == "register" else 0, no_cpu=True,
                              no_host=True,
                              gpus=world)
    r = bench.run_rank(args, rank, world, 0, dist, engine_cls=_StubEngine, device="cpu")
    if rank == 0:
        q.put(bench.report(args, r, world))
    dist.destroy_process_group()


@pytest.mark.parametrize("workload", ["sha256", "query", "register"])
def test_bench_two_ranks_gloo_scatter_gather(workload):
    """bench.run_rank over a 2-rank gloo group with the GPU path stubbed: rank 0 generates the job's
    inputs and scatters the shards, the ranks' statuses and public rows are gathered in global order,
    and the record reports n_gpus = 2. Also for the QueryIdentity and the config-3
    RegisterIdentityBuilder workloads (their rows)."""
    import hashlib
    import socket
    import torch.multiprocessing as mp
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bench_rank, args=(r, 2, port, q, workload)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=180)
    for p in ps:
        p.join(60)
    assert out["n_gpus"] == 2 and out["value"] > 0
    g = out["config"]["gathered"]
    if workload == "query":
        from pzkwit import query as Q
        rows = Q.batch_rows(12, seed=0x9, distinct=64)
    elif workload == "register":
        import bench
        rows = bench.make_register_inputs(12, 0, seed=bench.SIG_SEED[1], sig=1, workers=2)
    else:
        _, rows = I.sha256_config2_batch(12, seed=2, blocks=6)
    assert g["witnesses"] == 12
    assert g["status_nonzero"] == int((rows[:, 0, 0] != 0).sum())
    assert g["public_sha256"] == hashlib.sha256(rows[:, :4].tobytes()).hexdigest()[:16]
    assert out["config"]["invalid_lanes"] == 2 * int((rows[:, 0, 0] != 0).sum())
    if workload == "register":
        # the default register line also runs config 4's inputs (seed 0x4, proofs of depth 1-79) through the ranks
        c4 = out["config4"]
        rows4 = bench.make_register_inputs(12, 0, seed=4, sig=1, workers=2, smt_depth="1-79", smt_root=True)
        assert c4["n_gpus"] == 2 and c4["value"] > 0 and c4["smt_depth"] == "1-79"
        assert c4["invalid_lanes"] == 2 * int((rows4[:, 0, 0] != 0).sum())
    else:
        assert "config4" not in out


def test_sym_map_validation():
    """.sym maps (pzk_sym_check, the host half of pzk_instance_create_mapped): kept signals get dense
    witness indices; malformed, out-of-range, duplicate and gapped maps are rejected with a message."""
    from pzkwit import native, symmap
    n_o0 = native.layout_witness_size(I.CANONICAL)
    keep = symmap.synthetic_keep(n_o0, 1 + 4 + 5778)
    txt = symmap.sym_text(keep)
    assert native.sym_check(I.CANONICAL, txt) == int(keep[1:].sum()) + 1
    inv = symmap.parse_sym(txt)
    assert inv.shape[0] == int(keep[1:].sum()) + 1 and (np.diff(inv[1:]) > 0).all()
    # signals merged onto one witness index (circom --O1/--O2): accepted, the size is the number of indices
    merged = symmap.synthetic_keep(n_o0, 0, fraction=3, salt=0x77)
    txt2 = symmap.sym_text(keep, merged=merged)
    assert native.sym_check(I.CANONICAL, txt2) == int(keep[1:].sum()) + 1
    inv2 = symmap.parse_sym(txt2)
    assert (inv2 == inv).all()  # each index keeps its lowest signal
    assert native.sym_check(I.CANONICAL, "1,1,0,a\n2,1,0,b\n3,2,0,c\n") == 3
    for bad, msg in [("1,2,0,a\n", "not assigned"),
                     ("%d,1,0,a\n" % n_o0, "outside"), ("x,1,0,a\n", "expected"), ("1,-1,0,a\n", "no signal")]:
        with pytest.raises(native.PzkError, match=msg):
            native.sym_check(I.CANONICAL, bad)


# ---- config 5 (mixed flows) over two ranks: bench.run_mixed_rank with a stub engine and stub rows
def _mixed_row(gi, sg, n_in):
    """stub input row of global witness gi of flow sg: element k = (gi, sg, k) in its first bytes"""
    r = np.zeros((n_in, 32), dtype=np.uint8)
    k = np.arange(n_in)
    r[:, 0] = (gi * 7 + k) & 0xFF
    r[:, 1] = sg
    r[:, 2] = k & 0xFF
    r[:, 3] = k >> 8
    r[:, 4] = gi & 0xFF
    return r


def _mixed_stub_rows(sigs, lo, hi, n_in_max, workers):
    """bench._mixed_host_rows' layout (grouped per flow in MIX order, rows padded to n_in_max) with stub rows"""
    import bench
    from pzkwit import native
    out = np.zeros((hi - lo, n_in_max, 32), dtype=np.uint8)
    pos = 0
    for sg, idx in bench._mixed_groups(sigs, lo, hi).items():
        n_in = native.layout_inputs(dict(I.CANONICAL, sig=sg))
        for gi in idx:
            out[pos, :n_in] = _mixed_row(gi, sg, n_in)
            pos += 1
    return out


def _mixed_digest(row_bytes):
    import hashlib
    return np.frombuffer(hashlib.sha256(row_bytes).digest(), dtype=np.uint8)


class _MixedStubEngine:
    """bench.MixedGpuEngine's interface on the CPU. Status = element 0's byte 0 & 1 of the flow's compact row;
    public signals = elements 1..4 of the compact row and a digest of the WHOLE compact row (so a wrong per-flow
    width in the rank's cut shows)."""

    def __init__(self, flows, groups, dev):
        import torch
        from pzkwit import native
        self.torch, self.groups = torch, groups
        self.n_inputs = {sg: native.layout_inputs(flows[sg]) for sg in groups}

    def setup(self, d_in, first, n_local):
        self.d_in, self.first = d_in, first
        self.d_st = self.torch.zeros(n_local, dtype=self.torch.int32)

    def step(self):
        for sg in self.groups:
            rows = self.d_in[sg].view(-1, self.n_inputs[sg], 32)
            self.d_st[self.first[sg]: self.first[sg] + rows.shape[0]] = (rows[:, 0, 0] & 1).to(self.torch.int32)

    def sync(self):
        pass

    def statuses(self):
        return self.d_st

    def public_pass(self, n_pub):
        torch = self.torch
        pub = torch.zeros((self.d_st.shape[0], n_pub, 32), dtype=torch.uint8)
        for sg in self.groups:
            rows = self.d_in[sg].view(-1, self.n_inputs[sg], 32)
            f = self.first[sg]
            pub[f: f + rows.shape[0], :4] = rows[:, 1:5]
            for k in range(rows.shape[0]):
                pub[f + k, 4] = torch.from_numpy(_mixed_digest(rows[k].numpy().tobytes()).copy())
        return self.d_st.clone(), pub


def _mixed_rank(rank, world, port, q):
    import argparse
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = argparse.Namespace(workload="mixed", batch=10, steps=2, warmup=1, gpus=world)
    out = bench.run_mixed_rank(args, rank, world, 0, dist, engine_cls=_MixedStubEngine, device="cpu",
                               rows_fn=_mixed_stub_rows)
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def test_mixed_bench_two_ranks_gloo():
    """Config 5's multi-rank path (bench.run_mixed_rank) over a 2-rank gloo group with the GPU path stubbed: the
    per-flow grouped scatter from rank 0, each rank's cut back to compact rows of its flows' own widths, and the
    all-gather of statuses and public rows in rank-major, per-flow grouped order."""
    import hashlib
    import socket
    import torch.multiprocessing as mp
    import bench
    from pzkwit import native
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_mixed_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=180)
    for p in ps:
        p.join(60)
    assert out["n_gpus"] == 2 and out["value"] > 0
    # expected gather: rank-major, within a rank per flow (MIX order), global order inside a flow
    sigs, flows, costs, shards = bench._mixed_plan(10, 2)
    st, pub = [], []
    for lo, hi in shards:
        for sg, idx in bench._mixed_groups(sigs, lo, hi).items():
            n_in = native.layout_inputs(flows[sg])
            for gi in idx:
                r = _mixed_row(gi, sg, n_in)
                st.append(int(r[0, 0]) & 1)
                p = np.zeros((5, 32), dtype=np.uint8)
                p[:4] = r[1:5]
                p[4] = _mixed_digest(r.tobytes())
                pub.append(p)
    g = out["config"]["gathered"]
    assert g["witnesses"] == 20 and g["status_nonzero"] == sum(st)
    assert g["public_sha256"] == hashlib.sha256(np.stack(pub).tobytes()).hexdigest()[:16]
    assert out["config"]["invalid_lanes"] == sum(st)  # both ranks' last timed step
    assert set(out["config"]["flows"]) <= {"1", "2", "20"}


def test_mixed_engine_call_order(monkeypatch):
    """MixedGpuEngine issues a step's calls round robin over the flows, the flow with the largest witnesses first in
    every round (PZK_MIX_ORDER=flow: flow by flow); either way every row of every flow is covered exactly once."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    class E:
        pass
    e = E()
    e.groups = {1: list(range(1658)), 2: list(range(1246)), 20: list(range(1192))}
    e.sub = {1: 1156, 2: 898, 20: 420}
    e.witness_size = {1: 2251704, 2: 2828764, 20: 5488453}
    monkeypatch.delenv("PZK_MIX_ORDER", raising=False)
    rr = bench.MixedGpuEngine._calls(e)
    assert rr == [(20, 0), (2, 0), (1, 0), (20, 420), (2, 898), (1, 1156), (20, 840)]
    monkeypatch.setenv("PZK_MIX_ORDER", "flow")
    fl = bench.MixedGpuEngine._calls(e)
    assert fl == [(1, 0), (1, 1156), (2, 0), (2, 898), (20, 0), (20, 420), (20, 840)]
    for calls in (rr, fl):
        for sg, idx in e.groups.items():
            covered = sorted(r for g, a in calls if g == sg for r in range(a, min(a + e.sub[sg], len(idx))))
            assert covered == idx
