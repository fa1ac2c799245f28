"""GPU: streamed delivery into host memory (pzk_witness_stream, include/pzkwit.h; the batched form of
circuits/scripts/gen-witness.sh:25, which writes one .wtns per input). Every streamed row equals the
witness of the same passport from pzk_witness_batch_host, chunks arrive in order with their statuses, an
O0 and a .sym-mapped instance both stream, and a sink that stops the stream makes the call fail."""
import numpy as np
import pytest

from pzkwit import inputs as I, native, symmap

pytestmark = pytest.mark.gpu


def _rows(n, seed):
    g = I.PassportGen(seed=seed, n_keys=2, workers=1)
    rows = np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=i % 5)) for i in range(n)])
    rows[3, 0, 0] ^= 1  # slaveMerkleRoot changed: the SMT result is not enforced, the lane stays OK ...
    rows[4, 1, 0] = 2   # ... a non-bit message element flags its lane (PZK_ST_INPUT_RANGE or a range check)
    return rows


@pytest.mark.parametrize("mapped", [False, True])
def test_stream_rows_equal_host_batch(mapped):
    params = I.CANONICAL
    sym = None
    if mapped:
        keep = symmap.synthetic_keep(native.layout_witness_size(params), 1 + 4 + 5778, fraction=4)
        sym = symmap.sym_text(keep)
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params, sym=sym)
    rows = _rows(7, 0x5171 + mapped)
    want, want_st = inst.witness_batch_host(rows)
    assert want_st[4] != 0 and (np.delete(want_st, 4) == 0).all()
    got = np.zeros_like(want)
    got_st = np.full(len(rows), -1, dtype=np.int32)
    order = []

    def sink(first, w, st):
        order.append((first, w.shape[0]))
        got[first: first + w.shape[0]] = w
        got_st[first: first + w.shape[0]] = st

    inst.witness_stream(rows, sink, chunk=3)
    assert order == [(0, 3), (3, 3), (6, 1)]
    assert (got_st == want_st).all()
    for b in range(len(rows)):
        assert (got[b] == want[b]).all(), b
    # default chunking (~1 GiB of rows per chunk) in one call
    got2 = np.zeros_like(want)
    inst.witness_stream(rows, lambda first, w, st: got2.__setitem__(slice(first, first + w.shape[0]), w))
    assert (got2 == want).all()


def test_stream_sink_can_stop():
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL)
    rows = _rows(5, 0x5173)
    calls = []

    def sink(first, w, st):
        calls.append(first)
        return first >= 2  # stop after the second chunk

    with pytest.raises(native.PzkError, match="sink returned non-zero"):
        inst.witness_stream(rows, sink, chunk=2)
    assert calls == [0, 2]
    # the instance still works after a stopped stream
    w, st = inst.witness_batch_host(rows[:1])
    assert st[0] == 0 and w[0, 0, 0] == 1
