"""GPU, full size: the config-3 workload (BASELINE.json configs[2]) of 4096 canonical
RegisterIdentityBuilder passports, run through the device-resident C-ABI path the way bench.py runs it
(sub-batches into one reused output slab), and one GPU's 4096-row shard of config 4 (deep SMT
proofs), here with a ragged sub-batch of 1500 (1500, 1500, 1096 rows:
none a multiple of the 16-witness RSA groups or the 64-lane waves). The oracle cannot check 4096 rows of
72 MB in seconds, so the full batch is checked through size-independent properties:

* every lane's status is OK (every `===` check site of the circuit holds: RSA PKCS#1 signature, the
  hash chain of passportVerificationFlow, the SMT root, ...);
* witness[0] = 1 and passportHash (witness[2]) equals Poseidon(SHA-256(SA) low 252 bits) from hashlib;
* the rows repeat with period 1024 (1024 distinct passports tiled 4x), so row i and row i + 1024 —
  which sit at different offsets inside different sub-batches — must hold the same witness: their
  64-bit row checksums are compared for all 4096 rows;
* re-running the first sub-batch reproduces its checksums (determinism);
* sampled rows at the sub-batch edges are bit-exact against the CPU oracle.
"""
import hashlib

import numpy as np
import pytest

from pzkwit import field, inputs as I, native

pytestmark = pytest.mark.gpu

BATCH, DISTINCT, SUB = 4096, 1024, 1500

# config 3: shallow SMT proofs (depth 0..8); config 4 (BASELINE.json configs[3], "registerIdentity +
# depth-80 Sparse Merkle inclusion, batch 32768 over 8 GPUs"): one GPU's 4096-row shard of it, with
# proofs of depth 40..79, so every lane walks the upper half of SMTVerifier(80) up to its last level
FULLSIZE = {"config3": (3, lambda i: i % 9), "config4_shard": (4, lambda i: 40 + i % 40)}


@pytest.mark.parametrize("config", sorted(FULLSIZE))
def test_fullsize_properties(oracle, config):
    import torch
    params = I.CANONICAL
    seed, depth = FULLSIZE[config]
    g = I.PassportGen(seed=seed, n_keys=8, params=params, workers=1)
    pps = [g.passport_at(i, smt_depth=depth(i)) for i in range(DISTINCT)]
    rows = np.stack([I.pack_register_inputs(pp, params) for pp in pps])
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
    W, NIN = inst.witness_size, inst.n_inputs
    assert rows.shape == (DISTINCT, NIN, 32)

    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(np.tile(rows, (BATCH // DISTINCT, 1, 1))).to(dev)
    d_out = torch.empty((SUB, 32 * W), dtype=torch.uint8, device=dev)
    d_st = torch.empty(SUB, dtype=torch.int32, device=dev)
    one = torch.zeros(32, dtype=torch.uint8, device=dev)
    one[0] = 1
    sums = torch.empty(BATCH, dtype=torch.int64, device=dev)
    ph_expected = []
    for pp in pps:
        h = hashlib.sha256(pp["sa"]).digest()
        bits = [(h[i // 8] >> (7 - i % 8)) & 1 for i in range(252)]
        ph_expected.append(field.poseidon([sum(b << i for i, b in enumerate(bits))]))
    prm = oracle.register_params(**params)

    def run(lo, n):
        torch.cuda.synchronize()  # the library's streams do not wait for torch's stream
        inst.witness_batch_device(d_in.data_ptr() + lo * NIN * 32, n, d_out.data_ptr(), 32 * W, d_st.data_ptr(),
                                  device=0, sync=True)
        torch.cuda.synchronize()

    try:
        for lo in range(0, BATCH, SUB):
            n = min(SUB, BATCH - lo)
            run(lo, n)
            st = d_st[:n].cpu().numpy()
            assert (st == 0).all(), "lanes %s fail with %s" % (np.nonzero(st)[0][:8] + lo, st[st != 0][:8])
            assert bool((d_out[:n, :32] == one).all())
            ph = d_out[:n, 64:96].cpu().numpy()
            for r in range(n):
                assert int.from_bytes(ph[r].tobytes(), "little") == ph_expected[(lo + r) % DISTINCT], lo + r
            sums[lo:lo + n] = d_out[:n].view(torch.int64).sum(dim=1)
            for r in sorted({0, 1, n // 2, n - 1}):
                rc, ref = oracle.register_witness(prm, rows[(lo + r) % DISTINCT])
                assert rc == 0
                got = d_out[r].view(W, 32).cpu().numpy()
                bad = np.nonzero((ref != got).any(axis=1))[0]
                assert bad.size == 0, "row %d: %d elements differ, first %s" % (lo + r, bad.size, bad[:6])
        s = sums.view(BATCH // DISTINCT, DISTINCT)
        assert bool((s == s[0]).all()), "rows differ from their period-1024 copies"
        first = sums[:SUB].clone()
        run(0, SUB)
        assert bool((d_out.view(torch.int64).sum(dim=1) == first).all()), "re-run is not deterministic"
    finally:
        del d_out, d_in
        torch.cuda.empty_cache()


def test_pipelined_calls_match_serial_calls():
    """Calls issued back to back on the instance's own streams overlap (call k + 1's cores beside
    call k's emitters, alternating scratch sets; pzkwit.h pzk_exec.stream): five unsynchronised
    calls of ragged sizes into separate outputs give the same rows as one synchronised call each."""
    import torch
    params = I.CANONICAL
    g = I.PassportGen(seed=3, n_keys=4, params=params, workers=1)
    rows = np.stack([I.pack_register_inputs(g.passport_at(i, smt_depth=i % 5), params) for i in range(200)])
    inst = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
    W, NIN = inst.witness_size, inst.n_inputs
    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(rows).to(dev)
    cuts = [0, 37, 101, 102, 160, 200]
    d_out = torch.empty((200, 32 * W), dtype=torch.uint8, device=dev)
    d_st = torch.full((200,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # the library's streams do not wait for torch's stream
    try:
        for a, b in zip(cuts, cuts[1:]):
            inst.witness_batch_device(d_in.data_ptr() + a * NIN * 32, b - a, d_out[a].data_ptr(), 32 * W,
                                      d_st.data_ptr() + 4 * a)
        inst.sync()
        assert (d_st.cpu().numpy() == 0).all()
        piped = d_out.view(torch.int64).sum(dim=1)
        d_out.zero_()
        torch.cuda.synchronize()
        for a, b in zip(cuts, cuts[1:]):
            inst.witness_batch_device(d_in.data_ptr() + a * NIN * 32, b - a, d_out[a].data_ptr(), 32 * W,
                                      d_st.data_ptr() + 4 * a, sync=True)
        diff = torch.nonzero(d_out.view(torch.int64).sum(dim=1) != piped).flatten().tolist()
        assert not diff, "rows %s differ between pipelined and serial calls" % diff[:16]
    finally:
        del d_out, d_in
        torch.cuda.empty_cache()


def test_exec_device_mismatch_is_rejected():
    """pzk_exec.device must name the instance's device (pzkwit.h); the caller's current device is
    left as it was."""
    import torch
    inst = native.Instance(native.PZK_CIRCUIT_POSEIDON, 2)
    dev = torch.device("cuda:0")
    d_in = torch.zeros((1, inst.n_inputs, 32), dtype=torch.uint8, device=dev)
    d_out = torch.empty((1, 32 * inst.witness_size), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    with pytest.raises(native.PzkError, match="instance's device"):
        inst.witness_batch_device(d_in.data_ptr(), 1, d_out.data_ptr(), 32 * inst.witness_size, device=5)
    inst.witness_batch_device(d_in.data_ptr(), 1, d_out.data_ptr(), 32 * inst.witness_size, device=0, sync=True)
    assert torch.cuda.current_device() == 0
