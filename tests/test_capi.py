"""CPU: the C-ABI library loads, exports every entry point include/*.h declares, and its
host-side layout (no device needed) agrees with the oracle's independently derived sizes."""
import ctypes
import glob
import os
import re

import pytest

from pzkwit import inputs as I, native

HDRS = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "*.h")))


def declared_functions():
    src = "".join(open(h).read() for h in HDRS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pzk_\w+)\s*\(", src)))


def region_table(params):
    L = native.lib()
    p = native.PzkParams(circuit=native.PZK_CIRCUIT_REGISTER)
    for k, v in native.param_fields(params).items():
        setattr(p, k, v)
    info = native.PzkInfo()
    n = ctypes.c_uint32()
    assert L.pzk_layout_query(ctypes.byref(p), ctypes.byref(info), ctypes.byref(n)) == 0, L.pzk_last_error()
    out = []
    for i in range(n.value):
        off, ln, kd = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
        assert L.pzk_layout_region(ctypes.byref(p), i, ctypes.byref(off), ctypes.byref(ln), ctypes.byref(kd)) == 0
        out.append((off.value, ln.value, kd.value))
    return out


def layout_sizes(params, circuit=native.PZK_CIRCUIT_REGISTER, size_arg=0):
    L = native.lib()
    p = native.PzkParams(circuit=circuit, size_arg=size_arg)
    for k, v in native.param_fields(params or {}).items():
        setattr(p, k, v)
    info = native.PzkInfo()
    rc = L.pzk_layout_query(ctypes.byref(p), ctypes.byref(info), None)
    return rc, info.n_inputs, info.witness_size


def test_library_exports_header_symbols():
    L = native.lib()
    names = declared_functions()
    assert len(names) >= 12
    for nm in names:
        assert hasattr(L, nm), nm
    assert set(native.EXPORTS) <= set(names)
    assert L.pzk_version().startswith(b"pzkwit")


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    with pytest.raises(native.PzkError, match="no HIP device"):
        native.Instance(native.PZK_CIRCUIT_POSEIDON, 2)


@pytest.mark.parametrize("env,msg", [
    ({"PZK_BJJ": "bogus"}, "PZK_BJJ=bogus: valid values are rc, scratch"),
    ({"PZK_BJJ": "rc", "PZK_BJJ_SEGS": "8"}, "PZK_BJJ_SEGS=8: valid values are 16, 32, 64"),
    ({"PZK_BJJ_SEGS": "64"}, "PZK_BJJ_SEGS=64: valid values are 8, 16, 32"),  # the scratch core is the default
    ({"PZK_SHA_U": "7"}, "PZK_SHA_U=7: valid values are 8, 16, 32"),
])
def test_tuning_switches_validated(env, msg):
    """The tuning switches are checked before any device call (runtime.cpp pzk_instance_create): a bad value is an
    argument error on any host, GPU or not. Run in a child: the library reads the switches once per process."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from pzkwit import native\n"
            "try:\n    native.Instance(native.PZK_CIRCUIT_POSEIDON, 2)\nexcept native.PzkError as e:\n    print(e)\n"
            % os.path.dirname(os.path.dirname(native.__file__)))
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                         timeout=120)
    assert msg in out.stdout, out.stdout + out.stderr


PARAM_SETS = [
    I.CANONICAL,
    dict(I.CANONICAL, doc=1),                      # TD1 chunking (190-bit dg1 chunks)
    dict(I.CANONICAL, aa=0),                       # no active authentication
    dict(I.CANONICAL, ec_blocks=5, ec_shift=640),  # longer encapsulated content
    dict(I.CANONICAL, sig=2),                      # RSA-4096 (K = 64 limbs)
    dict(I.CANONICAL, sig=20),                     # ECDSA secp256r1
    dict(I.CANONICAL, sig=20, aa=0, doc=1),        # ECDSA, TD1, no AA
    dict(I.CANONICAL, sig=10),                     # RSA-PSS, e = 3, salt 32
    dict(I.CANONICAL, sig=11),                     # RSA-PSS, e = 65537, salt 32
    dict(I.CANONICAL, sig=12, aa=0),               # RSA-PSS, salt 64, no AA
    dict(I.CANONICAL, aa=2),                       # RSA AA key, DG15 checks scaled by 2
    dict(I.CANONICAL, aa=20),                      # EC AA key (256-bit field, 248 hashed bits)
    dict(I.CANONICAL, aa=22),                      # EC AA key, 320-bit field
    dict(I.CANONICAL, sig=20, aa=23),              # ECDSA signature, 192-bit EC AA key
    I.instance_params(13),                         # RSA-PSS SHA-384, salt 48, DG hash 384, 1024-bit blocks
    dict(I.instance_params(13), dg_hash=256, aa=0, dg15_blocks=0),  # SIG 13 with SHA-256 DG hashes, no DG15
    dict(I.instance_params(13), aa=20),            # SIG 13 with an EC AA key
    dict(I.CANONICAL, sig=21),                     # ECDSA brainpoolP256r1
    dict(I.CANONICAL, sig=14),                     # RSA-3072 PSS (K = 48: schoolbook BigMultOverflow)
    dict(I.CANONICAL, sig=3, dg_hash=160),         # RSA-2048 PKCS#1 v1.5 SHA-1, SHA-1 DG hashes
    dict(I.CANONICAL, sig=1, dg_hash=160, aa=0),   # SHA-1 DG hashes, SHA-256 signed attributes
    dict(I.CANONICAL, sig=4, dg_hash=160),         # RSA-3072 PKCS#1 v1.5 SHA-1, e = 37187 (20 BigMultModP)
    dict(I.CANONICAL, dg_hash=224),                # SHA-224 DG hashes
]


@pytest.mark.parametrize("params", PARAM_SETS)
def test_layout_sizes_match_oracle(oracle, params):
    rc, nin, nw = layout_sizes(params)
    assert rc == 0, native.lib().pzk_last_error()
    onin, onw = oracle.register_sizes(oracle.register_params(**params))
    assert (nin, nw) == (onin, onw)


@pytest.mark.parametrize("params", PARAM_SETS)
def test_regions_tile_the_witness(params):
    regs = sorted(region_table(params))
    pos = 0
    for off, ln, _ in regs:
        assert off == pos and ln > 0
        pos += ln
    assert pos == layout_sizes(params)[2]


def test_small_circuit_layouts(oracle):
    for n in range(1, 6):
        rc, nin, nw = layout_sizes(None, native.PZK_CIRCUIT_POSEIDON, n)
        assert rc == 0 and nin == n and nw == oracle.lib().orc_poseidon_witness_size(n)
    rc, nin, nw = layout_sizes(None, native.PZK_CIRCUIT_SHA256, 6)
    assert rc == 0 and nin == 3072 and nw == oracle.lib().orc_sha256_witness_size(6)
    for b in (1, 2, 4):
        rc, nin, nw = layout_sizes(None, native.PZK_CIRCUIT_SHA1, b)
        assert rc == 0 and nin == 512 * b and nw == oracle.lib().orc_sha1_witness_size(b)
    for circ, o in ((native.PZK_CIRCUIT_SHA384, 384), (native.PZK_CIRCUIT_SHA512, 512)):
        for b in (1, 2, 16):
            rc, nin, nw = layout_sizes(None, circ, b)
            assert rc == 0 and nin == 1024 * b and nw == oracle.lib().orc_sha512_witness_size(b, o)
        assert layout_sizes(None, circ, 0)[0] == -2 and layout_sizes(None, circ, 17)[0] == -2


def test_unsupported_params_rejected():
    rc, _, _ = layout_sizes(dict(I.CANONICAL, sig=22))  # brainpoolP320r1: not built yet
    assert rc == -2
    assert b"SIGNATURE_TYPE" in native.lib().pzk_last_error()
    # combinations the reference cannot compile (oracle params_ok agrees: test_oracle.py::test_pss384_oracle_sig13)
    assert layout_sizes(dict(I.CANONICAL, dg_hash=384))[0] == -2  # DG hash wider than the EC hash
    assert b"wider" in native.lib().pzk_last_error()
    assert layout_sizes(dict(I.instance_params(13), dg_hash=256))[0] == -2  # dg15 block sizes differ
    assert b"dg15 block sizes" in native.lib().pzk_last_error()
    rc, _, _ = layout_sizes(dict(I.CANONICAL, dg1_shift=2000))
    assert rc == -2


def test_wtns_header_layout():
    # 76 bytes: "wtns", v2, 2 sections; sec1 (n8=32, prime, witnessSize); sec2 header
    import struct
    from pzkwit.field import P
    hdr = bytearray(76)
    hdr[0:4] = b"wtns"
    # construct expected with a host-side writer and compare against the library's layout rules
    assert struct.calcsize("<4sII") + struct.calcsize("<IQI32sI") + struct.calcsize("<IQ") == 76
    assert P.to_bytes(32, "little")[:4] == bytes([0x01, 0x00, 0x00, 0xF0])


def test_code_objects_keep_return_addresses():
    """Every gfx950 code object in libpzkwit.so: no callable device function overwrites its return
    address (s[30:31]) before saving it. ROCm 7.2's branch relaxation can expand a far branch of a large
    callable function through those registers; the function then returns into its own body. This was the
    round-2 EC table walker hang / illegal access: the walker is force-inlined now, and
    this check keeps any later large callable function from reintroducing it."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import check_code_objects
    assert os.path.exists(native.LIB_PATH)
    assert check_code_objects.check(native.LIB_PATH) == []
