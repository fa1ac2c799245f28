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


def _host_pair(params, txt, rows):
    o0 = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
    mp = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params, sym=txt)
    w0, s0 = o0.witness_batch_host(rows)
    wm, sm = mp.witness_batch_host(rows)
    return w0, s0, wm, sm


@pytest.mark.parametrize("sig", [20, 13, 3, 11, 2])
def test_direct_mapped_emission_every_emitter(sig):
    """Monotone maps are emitted directly by every emitter (mapsink.hpp): ECDSA table blocks (k_emit_ect),
    SHA-384 (k_emit_sha512), SHA-1 (k_emit_sha1), RSA-PSS derived hashers, RSA-4096 BigMultModP (K = 64),
    plus the common SHA-256 / Poseidon / BigMultModP / BabyJubJub / small-region emitters. The map also
    merges signals onto shared witness indices (circom --O1/--O2). Mapped rows == the O0 rows at the kept
    indices, element for element."""
    params = I.instance_params(sig)
    keep = _keep(params, 3)
    merged = symmap.synthetic_keep(keep.shape[0], 0, fraction=7, salt=0x41)
    txt = symmap.sym_text(keep, merged=merged)
    inv = symmap.parse_sym(txt)
    g = I.PassportGen(seed=0x70 + sig, n_keys=1, params=params, workers=1)
    rows = np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=2 * i), params) for i in range(3)])
    w0, s0, wm, sm = _host_pair(params, txt, rows)
    assert (s0 == 0).all() and (sm == 0).all()
    assert wm.shape[1] == inv.shape[0]
    for b in range(rows.shape[0]):
        bad = np.nonzero((wm[b] != w0[b][inv]).any(axis=1))[0]
        assert bad.size == 0, "sig %d row %d: %d mapped elements differ (first k=%d, O0 %d)" % (
            sig, b, bad.size, bad[0], inv[bad[0]])


def test_keep_all_map_is_o0_and_nonmonotone_map_gathers():
    """A map that keeps every signal in order reproduces the O0 witness through the direct path; a map that
    is not monotone (two kept signals with swapped witness indices) takes the staging + gather path and is
    still the O0 witness at its indices."""
    params = I.CANONICAL
    n_o0 = native.layout_witness_size(params)
    g = I.PassportGen(seed=0x63, n_keys=1, workers=1)
    rows = np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=i)) for i in range(2)])
    w0, _, wm, sm = _host_pair(params, symmap.sym_text(np.ones(n_o0, dtype=bool)), rows)
    assert (sm == 0).all() and wm.shape == w0.shape and (wm == w0).all()
    keep = _keep(params, 5)
    lines = symmap.sym_text(keep).splitlines()
    kept = [i for i, ln in enumerate(lines) if int(ln.split(",")[1]) > 100]
    a, b = kept[10], kept[5000]
    la, lb = lines[a].split(","), lines[b].split(",")
    la[1], lb[1] = lb[1], la[1]
    lines[a], lines[b] = ",".join(la), ",".join(lb)
    txt = "\n".join(lines) + "\n"
    inv = symmap.parse_sym(txt)
    assert (np.diff(inv[1:]) < 0).any()
    _, _, wm2, sm2 = _host_pair(params, txt, rows)
    assert (sm2 == 0).all() and (wm2 == w0[:, inv]).all()


@pytest.mark.parametrize("name,level", [("register_canonical", 1), ("register_canonical", 2), ("register_sig20", 2),
                                        ("query", 1), ("query", 2)])
def test_shape_maps_equal_o0_subset(name, level):
    """The circom-shaped maps (approximate --O1 / --O2, data/shape/, tools/gen_shape_maps.py): every emitter writes
    only the kept elements (mapsink.hpp kept_collect / desc_run) and the mapped rows equal the O0 rows at the map's
    indices, element for element, with merged signals read through their class's first signal."""
    wit = symmap.load_shape(name, level)
    txt = symmap.sym_text_wit(wit)
    inv = symmap.parse_sym(txt)
    if name == "query":
        from pzkwit import query as Q
        from pzkwit.field import SplitMix64
        rng = SplitMix64(0x5A + level)
        rows = np.stack([Q.pack(Q.make_query(rng, depth=d)[0]) for d in (0, 79, 40, None, 5)])
        o0 = native.Instance(native.PZK_CIRCUIT_QUERY, 80)
        mp = native.Instance(native.PZK_CIRCUIT_QUERY, 80, sym=txt)
    else:
        params = I.CANONICAL if name == "register_canonical" else I.instance_params(20)
        g = I.PassportGen(seed=0x90 + level, n_keys=1, params=params, workers=1)
        rows = np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=3 * i), params) for i in range(3)])
        o0 = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
        mp = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params, sym=txt)
    assert mp.witness_size == inv.shape[0] == wit.max() + 1
    w0, s0 = o0.witness_batch_host(rows)
    wm, sm = mp.witness_batch_host(rows)
    assert (s0 == 0).all() and (sm == s0).all()
    for b in range(rows.shape[0]):
        bad = np.nonzero((wm[b] != w0[b][inv]).any(axis=1))[0]
        assert bad.size == 0, "%s O%d row %d: %d mapped elements differ (first k=%d, O0 %d)" % (
            name, level, b, bad.size, bad[0], inv[bad[0]])
        merged = np.flatnonzero(wit >= 0)
        assert (w0[b][merged] == wm[b][wit[merged]]).all()  # merged signals carry their class's value
