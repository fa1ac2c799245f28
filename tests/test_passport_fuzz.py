"""CPU: the EF.SOD parser (csrc/passport.cpp) reads untrusted DER, so it is run under AddressSanitizer +
UndefinedBehaviorSanitizer (tools/fuzz: the same source built for the host with -fsanitize) over
mutated SOD files — byte flips, truncations, length-byte edits, inserted and deleted bytes of the
reference-checked fixtures (tests/golden/sod_vectors.json). Every input must parse or be rejected
without a sanitizer report, and the unmutated files must parse to the reference's circuit names."""
import base64
import json
import os
import random
import shutil
import struct
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tools", "fuzz", "build", "passport_fuzz")
CASES = json.load(open(os.path.join(REPO, "tests", "golden", "sod_vectors.json")))["cases"]


@pytest.fixture(scope="module")
def fuzz_bin():
    if shutil.which("g++") is None:
        pytest.skip("no host C++ compiler")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tools", "fuzz")])
    return BIN


def record(dg1, dg15, sod):
    return b"".join(struct.pack("<I", len(x)) + x for x in (dg1, dg15, sod))


def mutate(sod, rng):
    b = bytearray(sod)
    op = rng.randrange(5)
    if op == 0:  # flip 1-4 bytes
        for _ in range(rng.randint(1, 4)):
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
    elif op == 1:  # truncate
        del b[rng.randrange(1, len(b)):]
    elif op == 2:  # rewrite a byte that follows a constructed / string tag (usually a length)
        tags = [i for i in range(len(b) - 1) if b[i] in (0x30, 0x31, 0x04, 0x03, 0x02, 0xA0)] or [0]
        i = min(rng.choice(tags) + 1, len(b) - 1)
        b[i] = rng.choice([0x00, 0x7F, 0x80, 0x81, 0x82, 0x84, 0x87, 0xFF, rng.randrange(256)])
    elif op == 3:  # insert a byte
        b.insert(rng.randrange(len(b)), rng.randrange(256))
    else:  # delete a byte
        del b[rng.randrange(len(b))]
    return bytes(b)


def test_mutated_sods_under_sanitizers(fuzz_bin):
    rng = random.Random(0x50D)
    blobs, expect = [], []
    for c in CASES:
        dg1, dg15, sod = (base64.b64decode(c[f]) for f in ("dg1", "dg15", "sod"))
        blobs.append(record(dg1, dg15, sod))
        expect.append("ok " + c["reference"]["name"])
        for _ in range(150):
            blobs.append(record(dg1, dg15, mutate(sod, rng)))
            expect.append(None)
            if rng.random() < 0.1:  # a corrupted DG15 (AA key) too
                blobs.append(record(dg1, mutate(dg15, rng) if dg15 else b"\x30", sod))
                expect.append(None)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_bin], input=b"".join(blobs), capture_output=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert b"runtime error" not in r.stderr and b"ERROR: AddressSanitizer" not in r.stderr, r.stderr.decode()[-3000:]
    lines = r.stdout.decode().splitlines()
    assert len(lines) == len(blobs)
    for got, want in zip(lines, expect):
        if want is not None:
            assert got == want
    assert sum(x == "err" for x in lines) > len(lines) // 4  # the mutations do reach the rejection paths


def _der_len(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def test_deeply_nested_der_is_rejected(fuzz_bin):
    """Untrusted DER nested far past any real EF.SOD (definite and indefinite lengths, nested
    constructed BIT STRINGs / OCTET STRINGs, and an encapsulation chain of primitive OCTET STRINGs
    each holding the next) must be rejected by the nesting cap, not overflow the parser's stack."""
    blobs = []
    for depth in (100, 5000, 50000):
        blobs.append(b"\x30\x80" * depth + b"\x00\x00" * depth)          # indefinite SEQUENCEs
        blobs.append(b"\x23\x80" * depth + b"\x00\x00" * depth)          # constructed BIT STRINGs
        blobs.append(b"\x24\x80" * depth + b"\x00\x00" * depth)          # constructed OCTET STRINGs
        inner = b"\x05\x00"
        for _ in range(min(depth, 2000)):                                 # definite SEQUENCEs
            inner = b"\x30" + _der_len(len(inner)) + inner
        blobs.append(inner)
        inner = b"\x05\x00"
        for _ in range(min(depth, 2000)):                                 # encapsulated OCTET STRINGs
            inner = b"\x04" + _der_len(len(inner)) + inner
        blobs.append(inner)
    c = CASES[0]
    dg1 = base64.b64decode(c["dg1"])
    data = b"".join(record(dg1, b"", sod) for sod in blobs) + b"".join(record(dg1, sod, base64.b64decode(c["sod"]))
                                                                       for sod in blobs[:5])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_bin], input=data, capture_output=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert b"runtime error" not in r.stderr and b"ERROR: AddressSanitizer" not in r.stderr, r.stderr.decode()[-3000:]
    lines = r.stdout.decode().splitlines()
    assert len(lines) == len(blobs) + 5
    assert all(x == "err" for x in lines), lines
