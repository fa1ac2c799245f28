"""GPU parity for the standalone circuits of configs 1 and 2:
PoseidonHash(n) and Sha256HashChunks(6). Every witness element is compared bit-for-bit
with the CPU oracle; SHA digests are also checked against hashlib."""
import hashlib
import json
import os

import numpy as np
import pytest

from pzkwit import field, inputs, native

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "poseidon_kats.json")


def elems(vals):
    return np.stack([np.frombuffer(int(v).to_bytes(32, "little"), dtype=np.uint8) for v in vals])


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5])
def test_poseidon_circuit_matches_oracle(oracle, n):
    inst = native.Instance(native.PZK_CIRCUIT_POSEIDON, n)
    rng = field.SplitMix64(0x100 + n)
    rows = [[rng.fr() for _ in range(n)] for _ in range(96)]
    rows[0] = [0] * n
    rows[1] = [field.P - 1] * n
    batch = np.stack([elems(r) for r in rows])
    wit, st = inst.witness_batch_host(batch)
    assert (st == 0).all()
    for b in range(len(rows)):
        rc, ref = oracle.poseidon_witness(rows[b])
        assert rc == 0
        assert ref.shape == wit[b].shape
        bad = np.nonzero((ref != wit[b]).any(axis=1))[0]
        assert bad.size == 0, "row %d: first mismatching signal %d" % (b, bad[0])


def test_poseidon_circuit_kats():
    d = json.load(open(GOLD))
    for n in (1, 2, 3, 4, 5):
        cases = [c for c in d["cases"] if len(c["in"]) == n]
        inst = native.Instance(native.PZK_CIRCUIT_POSEIDON, n)
        batch = np.stack([elems([int(x) for x in c["in"]]) for c in cases])
        wit, st = inst.witness_batch_host(batch)
        assert (st == 0).all()
        got = [int.from_bytes(wit[i, 1].tobytes(), "little") for i in range(len(cases))]
        assert got == [int(c["out"]) for c in cases]


def test_sha256_circuit_matches_oracle_and_hashlib(oracle):
    msgs, batch = inputs.sha256_config2_batch(64, seed=2, blocks=6)
    inst = native.Instance(native.PZK_CIRCUIT_SHA256, 6)
    wit, st = inst.witness_batch_host(batch)
    assert (st == 0).all()
    for b, m in enumerate(msgs):
        dig = np.packbits(wit[b, 1:257, 0]).tobytes()
        assert dig == hashlib.sha256(m).digest()
    for b in range(4):
        rc, ref = oracle.sha256_witness(batch[b], 6)
        assert rc == 0
        bad = np.nonzero((ref != wit[b]).any(axis=1))[0]
        assert bad.size == 0, "msg %d: first mismatching signal %d of %d" % (b, bad[0], ref.shape[0])


@pytest.mark.parametrize("blocks", [1, 3])
def test_sha1_circuit_matches_oracle_and_hashlib(oracle, blocks):
    """Sha1HashChunks(blocks) (hasher/sha1/sha1.circom:7-57) on the GPU: digests equal hashlib.sha1 and
    every one of the 198,034 signals per Sha1compression block equals the oracle's."""
    rng = np.random.default_rng(40 + blocks)
    msgs, rows = [], []
    for i in range(48):
        ln = int(rng.integers(64 * blocks - 72, 64 * blocks - 8))
        m = rng.integers(0, 256, max(ln, 0), dtype=np.uint8).tobytes()
        p = inputs.sha_pad(m)
        assert len(p) == 64 * blocks
        r = np.zeros((512 * blocks, 32), np.uint8)
        r[:, 0] = inputs.bits_msb_first(p)
        msgs.append(m)
        rows.append(r)
    batch = np.stack(rows)
    inst = native.Instance(native.PZK_CIRCUIT_SHA1, blocks)
    wit, st = inst.witness_batch_host(batch)
    assert (st == 0).all()
    for b, m in enumerate(msgs):
        assert np.packbits(wit[b, 1:161, 0]).tobytes() == hashlib.sha1(m).digest()
    for b in range(3):
        rc, ref = oracle.sha1_witness(batch[b], blocks)
        assert rc == 0
        bad = np.nonzero((ref != wit[b]).any(axis=1))[0]
        assert bad.size == 0, "msg %d: %d mismatching signals, first %s" % (b, bad.size, bad[:8].tolist())


@pytest.mark.parametrize("out_bits,blocks", [(384, 1), (512, 1), (384, 2), (512, 3)])
def test_sha512_circuit_matches_oracle_and_hashlib(oracle, out_bits, blocks):
    """Sha384HashChunks / Sha512HashChunks(blocks) (hasher/sha2/sha384/sha384HashChunks.circom:8-48,
    sha512/sha512HashChunks.circom) on the GPU: digests equal hashlib.sha384 / sha512, and every one of
    the 378,362 signals per Sha2_384_512 block (round sums up to 67 bits) equals the oracle's."""
    circ = native.PZK_CIRCUIT_SHA384 if out_bits == 384 else native.PZK_CIRCUIT_SHA512
    ref = hashlib.sha384 if out_bits == 384 else hashlib.sha512
    rng = np.random.default_rng(50 + out_bits + blocks)
    msgs, rows = [], []
    for i in range(40):
        ln = int(rng.integers(max(128 * blocks - 144, 0), 128 * blocks - 16))
        m = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        p = inputs.sha_pad(m, 1024)
        assert len(p) == 128 * blocks
        r = np.zeros((1024 * blocks, 32), np.uint8)
        r[:, 0] = inputs.bits_msb_first(p)
        msgs.append(m)
        rows.append(r)
    batch = np.stack(rows)
    inst = native.Instance(circ, blocks)
    wit, st = inst.witness_batch_host(batch)
    assert (st == 0).all()
    for b, m in enumerate(msgs):
        assert np.packbits(wit[b, 1:1 + out_bits, 0]).tobytes() == ref(m).digest(), b
    for b in range(3):
        rc, refw = oracle.sha512_witness(batch[b], blocks, out_bits)
        assert rc == 0
        assert refw.shape == wit[b].shape
        bad = np.nonzero((refw != wit[b]).any(axis=1))[0]
        assert bad.size == 0, "msg %d: %d mismatching signals, first %s" % (b, bad.size, bad[:8].tolist())


def test_sha512_circuit_rejects_nonbinary_input():
    """A message element outside {0, 1} fails the core's range check (status ST_INPUT_RANGE)."""
    r = np.zeros((2, 1024, 32), np.uint8)
    r[1, 5, 0] = 2
    inst = native.Instance(native.PZK_CIRCUIT_SHA512, 1)
    _, st = inst.witness_batch_host(r)
    assert st[0] == 0 and st[1] != 0


def test_sha256_config2_fullsize(oracle):
    """Config 2 at its stated size (BASELINE.json configs[1]): Sha256HashChunks(6),
    batch 1024, seed 2, on the device-buffer path. All 1024 digests equal hashlib.sha256; rows 0, 1,
    511, 1023 are bit-exact against the oracle; a re-run reproduces every row's checksum."""
    import torch
    n = 1024
    msgs, rows = inputs.sha256_config2_batch(n, seed=2, blocks=6)
    inst = native.Instance(native.PZK_CIRCUIT_SHA256, 6)
    W, NIN = inst.witness_size, inst.n_inputs
    assert rows.shape == (n, NIN, 32)
    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(rows).to(dev)
    d_out = torch.empty((n, W * 32), dtype=torch.uint8, device=dev)
    d_st = torch.full((n,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # the library's streams do not wait for torch's stream
    try:
        inst.witness_batch_device(d_in.data_ptr(), n, d_out.data_ptr(), 32 * W, d_st.data_ptr(), sync=True)
        assert (d_st.cpu().numpy() == 0).all()
        bits = d_out.view(n, W, 32)[:, 1:257, 0].cpu().numpy()
        for b, m in enumerate(msgs):
            assert np.packbits(bits[b]).tobytes() == hashlib.sha256(m).digest(), b
        for b in (0, 1, 511, 1023):
            rc, ref = oracle.sha256_witness(rows[b], 6)
            assert rc == 0
            got = d_out[b].view(W, 32).cpu().numpy()
            bad = np.nonzero((ref != got).any(axis=1))[0]
            assert bad.size == 0, "msg %d: first mismatching signal %d" % (b, bad[0])
        sums = d_out.view(torch.int64).sum(dim=1)
        d_out.zero_()
        torch.cuda.synchronize()
        inst.witness_batch_device(d_in.data_ptr(), n, d_out.data_ptr(), 32 * W, d_st.data_ptr(), sync=True)
        assert bool((d_out.view(torch.int64).sum(dim=1) == sums).all()), "re-run is not deterministic"
    finally:
        del d_out, d_in
        torch.cuda.empty_cache()
