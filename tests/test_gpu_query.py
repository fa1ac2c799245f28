"""QueryIdentity(80) on the GPU: every element of every witness bit-exact against the
CPU oracle (oracle/query.inc.c), lane statuses equal to the oracle's check sites, and a full 4096-witness
batch with its public outputs checked against independent math."""
import numpy as np
import pytest

from pzkwit import native, query as Q
from pzkwit.field import SplitMix64

from test_query import FAIL_KINDS, _fail_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def inst():
    return native.Instance(native.PZK_CIRCUIT_QUERY, 80)


@pytest.fixture(scope="module")
def inst_td1():
    return native.Instance(native.PZK_CIRCUIT_QUERY, 80, {"doc": 1})


def _compare(oracle, rows, wit, st, codes, td1=False):
    for b in range(rows.shape[0]):
        rc, ref = oracle.query_witness(rows[b], td1=td1)
        assert rc == codes[b] == st[b], (b, rc, codes[b], st[b])
        bad = np.nonzero((ref != wit[b]).any(axis=1))[0]
        assert bad.size == 0, "row %d: %d mismatching signals, first %d" % (b, bad.size, bad[0])


@pytest.mark.parametrize("td1", [False, True])
def test_query_matches_oracle(oracle, inst, inst_td1, td1):
    I = inst_td1 if td1 else inst
    assert I.witness_size == oracle.query_sizes(td1)[1] and I.n_inputs == (Q.N_INPUTS_TD1 if td1 else Q.N_INPUTS)
    rng = SplitMix64(0x5151 + td1)
    rows, codes = [], []
    for k in range(40):
        sel = [0, (1 << 18) - 1, None, None][k % 4]
        depth = [0, 1, 79, 40, None][k % 5]
        inp, _ = Q.make_query(rng, selector=sel, depth=depth, td1=td1)
        rows.append(Q.pack(inp))
        codes.append(0)
    for i, kind in enumerate(FAIL_KINDS):  # one failing lane per check site, between valid ones
        inp, code = _fail_case(kind, SplitMix64(0x77 + i), td1)
        rows.insert(3 * i + 1, Q.pack(inp))
        codes.insert(3 * i + 1, code)
    rows = np.stack(rows)
    wit, st = I.witness_batch_host(rows)
    _compare(oracle, rows, wit, st, codes, td1)


def test_query_full_batch(oracle, inst):
    """4096 witnesses (64 distinct queries tiled) in one call: every lane passes, every lane's public outputs
    equal independent math, repeated rows are identical, and rows at the batch edges equal the oracle."""
    rng = SplitMix64(0x4096)
    uniq = [Q.make_query(rng) for _ in range(64)]
    rows = np.stack([Q.pack(inp) for inp, _ in uniq])
    batch = np.concatenate([rows] * 64)
    wit, st = inst.witness_batch_host(batch)
    assert (st == 0).all()
    for i in range(4096):
        inp, info = uniq[i % 64]
        got = [int.from_bytes(wit[i, 1 + k].tobytes(), "little") for k in range(9)]
        assert got == Q.public_outputs(inp, info), i
    assert (wit[:64] == wit[4032:]).all()
    _compare(oracle, batch[[0, 63, 4095]], wit[[0, 63, 4095]], st[[0, 63, 4095]], [0, 0, 0])


@pytest.mark.parametrize("td1", [False, True])
def test_query_device_witnesses_satisfy_constraints(inst, inst_td1, td1):
    """Device witnesses through the independent constraint checker (oracle/r1cs_query.inc.c): every constraint
    holds and every signal is read by one."""
    import pyr1cs
    rng = SplitMix64(0xC1)
    rows = np.stack([Q.pack(Q.make_query(rng, selector=s, depth=d, td1=td1)[0])
                     for s, d in ((0, 0), ((1 << 18) - 1, 79), (None, 40), (None, None))])
    wit, st = (inst_td1 if td1 else inst).witness_batch_host(rows)
    assert (st == 0).all()
    for b in range(rows.shape[0]):
        rc, rep = pyr1cs.check_query(wit[b], td1=td1)
        assert rc == 0 and rep["n_failed"] == 0 and rep["n_uncovered"] == 0, (b, rep)


def test_query_witness_calculator_json(oracle):
    """The reference-shaped surface (WitnessCalculator.calculateWitness over the circuit's JSON signal names)
    on a query: equals the oracle's witness."""
    from pzkwit import witness_calculator
    wc = witness_calculator.WitnessCalculator(native.PZK_CIRCUIT_QUERY, 80)
    inp, _ = Q.make_query(SplitMix64(0x3E), selector=(1 << 18) - 1)
    w = wc.calculateWitness({k: (v if isinstance(v, list) else str(v)) for k, v in inp.items()}, True)
    rc, ref = oracle.query_witness(Q.pack(inp))
    assert rc == 0 and len(w) == ref.shape[0]
    assert all(w[i] == int.from_bytes(ref[i].tobytes(), "little") for i in range(len(w)))


def _nonmonotone_query_map(n_o0, n_in):
    """A query .sym map that keeps a third of the signals and swaps two kept witness indices, so the instance
    takes the staging + gather path (runtime.cpp batch_mapped)."""
    from pzkwit import symmap
    lines = symmap.sym_text(symmap.synthetic_keep(n_o0, 1 + 9 + n_in, fraction=3)).splitlines()
    kept = [i for i, ln in enumerate(lines) if int(ln.split(",")[1]) > 20]
    a, b = kept[7], kept[len(kept) // 2]
    la, lb = lines[a].split(","), lines[b].split(",")
    la[1], lb[1] = lb[1], la[1]
    lines[a], lines[b] = ",".join(la), ",".join(lb)
    txt = "\n".join(lines) + "\n"
    inv = symmap.parse_sym(txt)
    assert (np.diff(inv[1:]) < 0).any()
    return txt, inv


def test_query_gathered_map_over_three_chunks_and_stream(inst):
    """QueryIdentity calls rotate their chain over three streams (runtime.cpp batch_locked); a gathered map runs a
    batch as chunks of 1024 witnesses through two O0 staging slots. 2200 witnesses = three chunks, so chunk 3
    reuses chunk 1's slot while chunk 2's chain runs on another stream: every row must equal the O0 witness at the
    map's indices, through witness_batch_host and through witness_stream (inputs uploaded on the stream's own
    stream)."""
    rng = SplitMix64(0x3C3)
    uniq = np.stack([Q.pack(Q.make_query(rng, depth=[0, 79, 40, None][k % 4])[0]) for k in range(40)])
    w0, s0 = inst.witness_batch_host(uniq)
    assert (s0 == 0).all()
    txt, inv = _nonmonotone_query_map(inst.witness_size, inst.n_inputs)
    mp = native.Instance(native.PZK_CIRCUIT_QUERY, 80, sym=txt)
    assert mp.witness_size == inv.shape[0]
    n = 2200
    rows = np.concatenate([uniq] * (n // 40))
    want = w0[:, inv]
    wm, sm = mp.witness_batch_host(rows)
    assert (sm == 0).all()
    for i in range(0, n, 97):
        assert (wm[i] == want[i % 40]).all(), i
    assert all((wm[i] == want[i % 40]).all() for i in range(n - 40, n))
    del wm
    seen = []

    def sink(first, w, st):
        assert (st == 0).all()
        for k in range(0, w.shape[0], 61):
            assert (w[k] == want[(first + k) % 40]).all(), first + k
        assert (w[-1] == want[(first + w.shape[0] - 1) % 40]).all()
        seen.append((first, w.shape[0]))

    mp.witness_stream(rows, sink, chunk=n)
    assert seen == [(0, n)]
