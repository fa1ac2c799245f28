"""CPU: the CPU restatement (oracle/witness_oracle.c) and the constraint checker (oracle/r1cs_check.c) built
with -fsanitize=address,undefined (`make -C oracle san`, oracle/san_main.c) over register witnesses of the
RSA PKCS#1 v1.5, RSA-PSS (SHA-256 / SHA-384) and ECDSA instances and over the standalone SHA-256 / SHA-1 /
SHA-384 / Poseidon circuits: every case evaluates, satisfies its constraints, and the sanitizers report
nothing (host ASan/UBSan build of the CPU restatement). Test infrastructure checking test
infrastructure: the product path (the HIP library) is not involved."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from pzkwit import field, inputs as I

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "oracle", "build", "san_main")
DATA = os.path.join(REPO, "passport-zk-circuits_amd", "data")
KEYS = ("sig", "dg_hash", "doc", "ec_blocks", "ec_shift", "dg1_shift", "aa", "dg15_shift", "dg15_blocks", "aa_shift")


def _record(kind, params, rows):
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    return struct.pack("<i10ii", kind, *params, rows.shape[0]) + rows.tobytes()


@pytest.fixture(scope="module")
def san_main():
    if shutil.which(os.environ.get("CC", "gcc")) is None:
        pytest.skip("no C compiler")
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "san"], capture_output=True, text=True)
    if r.returncode != 0:
        if "asan" in r.stderr.lower() or "ubsan" in r.stderr.lower():
            pytest.skip("toolchain without sanitizer runtimes: " + r.stderr[-300:])
        raise AssertionError(r.stderr)
    return SAN


def test_sanitized_oracle_and_checker(san_main, tmp_path):
    recs = []
    for params, depth in ((dict(I.CANONICAL), 3), (I.instance_params(13), 0), (I.instance_params(20), 1),
                          (dict(I.CANONICAL, doc=1, aa=20), 0)):
        g = I.PassportGen(seed=0x5A, n_keys=1, params=params, workers=1)
        pp = g.passport_at(0, smt_depth=depth)
        if pp["root"] is None:
            pp["root"] = field.SplitMix64(7).fr()
        recs.append(_record(0, [params[k] for k in KEYS], I.pack_register_inputs(pp, params)))
    _, rows = I.sha256_config2_batch(1, seed=2, blocks=6)
    recs.append(_record(1, [6] + [0] * 9, rows[0]))
    for kind, bits, blk, nbits in ((2, 512, 2, 0), (3, 1024, 2, 384)):
        m = bytes(range(blk * bits // 8 - 40))
        r = np.zeros((bits * blk, 32), np.uint8)
        r[:, 0] = I.bits_msb_first(I.sha_pad(m, bits))
        recs.append(_record(kind, [blk, nbits] + [0] * 8, r))
    for n in (1, 5):
        rng = field.SplitMix64(n)
        r = np.stack([np.frombuffer(rng.fr().to_bytes(32, "little"), np.uint8) for _ in range(n)])
        recs.append(_record(4, [n] + [0] * 9, r))
    cases = tmp_path / "cases.bin"
    cases.write_bytes(b"".join(recs))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
    r = subprocess.run([san_main, DATA, str(cases)], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == len(recs), r.stdout
    for ln in lines:
        f = ln.split()
        assert f[5] == "0" and f[7] == "0" and f[9] == "0" and f[11] == "0", ln
