"""GPU: instances with a signal -> witness map (.sym, pzk_instance_create_mapped; VERDICT row N1). The
mapped witness must be exactly the O0 witness restricted to the kept signals in witness-index order:
checked against the oracle's O0 vector (one passport, host path) and against an O0 instance on the
device for a 300-passport batch (two internal chunks of the mapped path, ragged)."""
import numpy as np
import pytest

from pzkwit import inputs as I, native, symmap

pytestmark = pytest.mark.gpu


def _keep(params, fraction):
    n_o0 = native.layout_witness_size(params)
    n_in = I.PassportGen(seed=3, n_keys=1, params=params, workers=1).n_inputs
    return symmap.synthetic_keep(n_o0, 1 + 4 + n_in, fraction=fraction)


def test_mapped_witness_equals_oracle_subset(oracle):
    params = I.CANONICAL
    keep = _keep(params, 3)
    txt = symmap.sym_text(keep)
    inv = symmap.parse_sym(txt)
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params, sym=txt)
    assert inst.witness_size == inv.shape[0]
    hdr = inst.wtns_header()
    assert int.from_bytes(hdr[60:64], "little") == inv.shape[0]  # wtns v2: witnessSize after n8 and the prime
    g = I.PassportGen(seed=0x61, n_keys=2, workers=1)
    rows = np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=0)) for i in range(2)])
    wit, st = inst.witness_batch_host(rows)
    assert (st == 0).all()
    for b in range(2):
        rc, ref = oracle.register_witness(oracle.register_params(**params), rows[b])
        assert rc == 0
        assert (wit[b] == ref[inv]).all()


def test_mapped_batch_equals_o0_batch_on_device():
    import torch
    params = I.CANONICAL
    keep = _keep(params, 4)
    txt = symmap.sym_text(keep)
    inv = torch.from_numpy(symmap.parse_sym(txt)).cuda()
    g = I.PassportGen(seed=0x62, n_keys=2, workers=1)
    base = np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=i % 4)) for i in range(20)])
    n = 300
    rows = np.tile(base, (n // 20, 1, 1))
    o0 = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
    mp = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params, sym=txt)
    W0, Wm = o0.witness_size, mp.witness_size
    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(rows).to(dev)
    out0 = torch.empty((n, W0, 32), dtype=torch.uint8, device=dev)
    outm = torch.empty((n, Wm, 32), dtype=torch.uint8, device=dev)
    st0 = torch.full((n,), -1, dtype=torch.int32, device=dev)
    stm = torch.full((n,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    try:
        o0.witness_batch_device(d_in.data_ptr(), n, out0.data_ptr(), 32 * W0, st0.data_ptr(), sync=True)
        mp.witness_batch_device(d_in.data_ptr(), n, outm.data_ptr(), 32 * Wm, stm.data_ptr(), sync=True)
        assert bool((st0 == 0).all()) and bool((stm == 0).all())
        for lo in range(0, n, 50):
            assert bool((out0[lo:lo + 50][:, inv] == outm[lo:lo + 50]).all()), lo
    finally:
        del out0, outm, d_in
        torch.cuda.empty_cache()
