"""GPU: device witnesses satisfy every constraint of the circuit (oracle/r1cs_check.c, the restated
checkConstraints of test/automatisationTest.js:51) — configs 1-5 through the C-ABI.
Independent of the element-for-element oracle comparison of the other GPU tests: the checker never
computes a witness value, it evaluates the templates' constraints on what the device wrote."""
import numpy as np
import pytest

from pzkwit import field, inputs as I, native

pytestmark = pytest.mark.gpu
pyr1cs = pytest.importorskip("pyr1cs")
from test_r1cs import expected_uncovered  # noqa: E402


def _ok(res, uncovered):
    rc, r = res
    assert r["oob"] == 0 and r["n_failed"] == 0 and r["n_uncovered_nonzero"] == 0, r
    assert r["n_uncovered"] == uncovered and rc == 0, r


def test_config1_poseidon_device_witnesses():
    for n in (1, 2, 3, 4, 5):
        rng = field.SplitMix64(0x900 + n)
        rows = np.stack([np.stack([np.frombuffer(rng.fr().to_bytes(32, "little"), np.uint8) for _ in range(n)])
                         for _ in range(8)])
        wit, st = native.Instance(native.PZK_CIRCUIT_POSEIDON, n).witness_batch_host(rows)
        assert (st == 0).all()
        for w in wit:
            _ok(pyr1cs.check_poseidon(w, n), 0)


def test_config2_sha256_device_witnesses():
    _, rows = I.sha256_config2_batch(24, seed=2, blocks=6)
    wit, st = native.Instance(native.PZK_CIRCUIT_SHA256, 6).witness_batch_host(rows)
    assert (st == 0).all()
    for w in wit:
        _ok(pyr1cs.check_sha256(w, 6), 0)


@pytest.mark.parametrize("out_bits,blocks", [(384, 2), (512, 1)])
def test_sha512_device_witnesses(out_bits, blocks):
    """Sha384HashChunks / Sha512HashChunks device witnesses (k_emit_sha512) satisfy every constraint."""
    rng = np.random.default_rng(out_bits + blocks)
    rows = []
    for _ in range(6):
        m = rng.integers(0, 256, int(rng.integers(128 * blocks - 120, 128 * blocks - 17)), dtype=np.uint8).tobytes()
        r = np.zeros((1024 * blocks, 32), np.uint8)
        r[:, 0] = I.bits_msb_first(I.sha_pad(m, 1024))
        rows.append(r)
    circ = native.PZK_CIRCUIT_SHA384 if out_bits == 384 else native.PZK_CIRCUIT_SHA512
    wit, st = native.Instance(circ, blocks).witness_batch_host(np.stack(rows))
    assert (st == 0).all()
    for w in wit:
        _ok(pyr1cs.check_sha512(w, blocks, out_bits), 0)


@pytest.mark.parametrize("sig,depths", [(1, [0, 1, 2, 40, 79, 0, 5, 17]), (2, [0, 9, 33]), (3, [0, 4]), (4, [2]),
                                        (10, [0, 3]), (11, [0, 6]), (12, [1]), (13, [0, 3]), (14, [0]), (20, [0, 2]),
                                        (21, [1]), (24, [0]), (25, [2])])
def test_config3_4_register_device_witnesses(sig, depths):
    """Config 3 (canonical, SMT root of the one-leaf tree) and config 4 (depth-k SMT paths), the
    RSA-4096 flow of config 5, the SHA-1 / RSA-3072 / RSA-PSS instances and the ECDSA curves (P-256,
    brainpoolP256r1, secp224r1, brainpoolP384r1): every device witness
    satisfies all of its constraints (2.25 M for the canonical instance)."""
    params = I.instance_params(sig)
    g = I.PassportGen(seed=0x40 + sig, n_keys=2, params=params, workers=1)
    pps = []
    for i, d in enumerate(depths):
        pp = g.passport_at(i, smt_depth=d)
        if pp["root"] is None:
            pp["root"] = field.SplitMix64(i).fr()
        pps.append(pp)
    rows = np.stack([I.pack_register_inputs(pp, params) for pp in pps])
    wit, st = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params).witness_batch_host(rows)
    assert (st == 0).all(), st
    for w in wit:
        _ok(pyr1cs.check_register(w, **params), expected_uncovered(sig))


def test_failing_lane_violates_constraints():
    """A lane whose signature does not verify is flagged by the device (lane status) and its witness
    violates the constraints; its neighbours' witnesses satisfy them."""
    g = I.PassportGen(seed=0x44, n_keys=2, workers=1)
    pps = [g.passport_at(i) for i in range(3)]
    pps[1]["sig"] = (pps[1]["sig"] + 1) % pps[1]["n"]
    rows = np.stack([I.pack_register_inputs(pp) for pp in pps])
    wit, st = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, I.CANONICAL).witness_batch_host(rows)
    assert st[0] == 0 and st[2] == 0 and st[1] != 0
    for b in (0, 2):
        _ok(pyr1cs.check_register(wit[b], **I.CANONICAL), 17 * 992)
    rc, r = pyr1cs.check_register(wit[1], **I.CANONICAL)
    assert rc != 0 and r["n_failed"] > 0
