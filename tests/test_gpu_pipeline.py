"""GPU: the scheduling paths of calls left in flight (runtime.cpp batch_locked / ensure_chain_streams), each
against the CPU oracle rather than against another run of the same code:

* two register instances on one device, so both take the reduced stream set (low-priority SMT chain streams, no
  post-chain stream); calls alternate between them without synchronising, then one instance is destroyed and the
  other's next calls drain and rebuild its stream set (the full one);
* an O2-shaped mapped instance (a monotone .sym keeping a quarter of the signals: odd calls' SHA emission on the
  second SHA stream) with back-to-back unsynchronised calls;
* QueryIdentity(80) with more calls in flight than it has scratch sets' worth of chain streams (six sets over four
  chain streams): eight unsynchronised calls.

Rows of every call are compared element for element with the oracle (sampled rows of each call)."""
import numpy as np
import pytest

from pzkwit import inputs as I, native, query as Q, symmap
from pzkwit.field import SplitMix64

pytestmark = pytest.mark.gpu


def _register_rows(seed, n, depth):
    g = I.PassportGen(seed=seed, n_keys=2, params=I.CANONICAL, workers=1)
    return np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=depth(i)), I.CANONICAL) for i in range(n)])


def _check_rows(oracle, rows, out, st, picks, inv=None):
    prm = oracle.register_params(**I.CANONICAL)
    for r in picks:
        rc, ref = oracle.register_witness(prm, rows[r])
        assert rc == 0 and st[r] == 0, (r, rc, st[r])
        want = ref if inv is None else ref[inv]
        bad = np.nonzero((want != out[r]).any(axis=1))[0]
        assert bad.size == 0, "row %d: %d elements differ, first %s" % (r, bad.size, bad[:6])


def _calls(torch, insts, rows, n_calls, per_call):
    """n_calls unsynchronised calls, round-robin over insts, each into its own output rows; -> [(inst, lo, out, st)]"""
    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(rows).to(dev)
    NIN = rows.shape[1]
    bufs = [(torch.empty((per_call, insts[k % len(insts)].witness_size, 32), dtype=torch.uint8, device=dev),
             torch.full((per_call,), -1, dtype=torch.int32, device=dev)) for k in range(n_calls)]
    done = []
    torch.cuda.synchronize()  # the library's streams do not wait for torch's stream (the buffers' fills)
    for k in range(n_calls):
        inst = insts[k % len(insts)]
        W = inst.witness_size
        lo = (k * per_call) % rows.shape[0]
        out, st = bufs[k]
        inst.witness_batch_device(d_in.data_ptr() + lo * NIN * 32, per_call, out.data_ptr(), 32 * W, st.data_ptr())
        done.append((inst, lo, out, st))
    for inst in insts:
        inst.sync()
    return [(inst, lo, out.cpu().numpy(), st.cpu().numpy()) for inst, lo, out, st in done], d_in


def test_two_register_instances_share_the_device(oracle):
    import torch
    rows = _register_rows(0x6A, 96, lambda i: (7 * i) % 80)
    a = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL)
    b = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL)
    res, d_in = _calls(torch, [a, b], rows, 6, 32)
    for inst, lo, out, st in res:
        _check_rows(oracle, rows[lo:lo + 32], out, st, [0, 31])
    # b goes away: a's next calls find it alone on the device and rebuild its stream set
    del b, res
    res, d_in = _calls(torch, [a], rows, 4, 24)
    for inst, lo, out, st in res:
        _check_rows(oracle, rows[lo:lo + 24], out, st, [0, 23])
    del d_in
    torch.cuda.empty_cache()


def test_o2_shaped_back_to_back_calls(oracle):
    import torch
    wit = symmap.load_shape("register_canonical", 2)
    txt = symmap.sym_text_wit(wit)
    inv = symmap.parse_sym(txt)
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL, sym=txt)
    assert 2 * inst.witness_size <= native.layout_witness_size(I.CANONICAL)  # the two-SHA-stream case
    rows = _register_rows(0x6B, 80, lambda i: (11 * i) % 80)
    res, d_in = _calls(torch, [inst], rows, 5, 16)
    for _, lo, out, st in res:
        _check_rows(oracle, rows[lo:lo + 16], out, st, [0, 7, 15], inv=inv)
    del d_in
    torch.cuda.empty_cache()


def test_query_eight_calls_in_flight(oracle):
    import torch
    inst = native.Instance(native.PZK_CIRCUIT_QUERY, 80)
    rng = SplitMix64(0x6C)
    rows = np.stack([Q.pack(Q.make_query(rng, depth=[0, 1, 40, 79, None][i % 5])[0]) for i in range(128)])
    res, d_in = _calls(torch, [inst], rows, 8, 16)
    for _, lo, out, st in res:
        assert (st == 0).all()
        for r in (0, 5, 15):
            rc, ref = oracle.query_witness(rows[lo + r])
            assert rc == 0
            bad = np.nonzero((ref != out[r]).any(axis=1))[0]
            assert bad.size == 0, "call at %d row %d: %d elements differ" % (lo, r, bad.size)
    del d_in
    torch.cuda.empty_cache()
