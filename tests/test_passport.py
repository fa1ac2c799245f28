"""CPU: the bulk SOD preprocessor (include/pzkpassport.h, csrc/passport.cpp) against the reference's own
processPassport (test/process_passport.js:674-816), run on Node 12 over synthetic EF.SOD files
(tests/golden/sod_vectors.json, tools/gen_sod_fixtures.*): the RegisterIdentityBuilder arguments
writeToCircom writes, the circuit name, and every input array writeToJson writes, element for element."""
import base64
import json
import os

import numpy as np
import pytest

from pzkwit import native, passport as PP
from pzkwit.field import P

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sod_vectors.json")
CASES = json.load(open(GOLDEN))["cases"]
ARGS = ("sig", "dg_hash", "doc", "ec_blocks", "ec_shift", "dg1_shift", "aa", "dg15_shift", "dg15_blocks", "aa_shift")


def src(c):
    return {f: c[f] for f in ("dg1", "dg15", "sod")}


def reference_row(ref, params, n_inputs):
    """The flat input row of the reference's input JSON (pack order of pzkwit.inputs.pack_register_inputs)."""
    j = ref["inputs"]
    row = np.zeros((n_inputs, 32), dtype=np.uint8)
    o = 0

    def put_int(v):
        nonlocal o
        row[o] = np.frombuffer(int(v % P).to_bytes(32, "little"), dtype=np.uint8)
        o += 1

    def put_bits(s):
        nonlocal o
        row[o:o + len(s), 0] = np.frombuffer(s.encode(), dtype=np.uint8) - 48
        o += len(s)

    put_int(int(j["slaveMerkleRoot"], 16))
    for f in ("encapsulatedContent", "dg1", "dg15", "signedAttributes"):
        put_bits(j[f])
    for f in ("signature", "pubkey"):
        for v in j[f]:
            row[o, :8] = np.frombuffer(int(v).to_bytes(8, "little"), dtype=np.uint8)
            o += 1
    o += j["branches"]
    put_int(int(j["skIdentity"], 16))
    assert o == n_inputs
    return row


@pytest.mark.parametrize("c", CASES, ids=lambda c: "sig%d_%d_%s" % (c["sig"], c["index"], "_".join(sorted(c["options"]))))
def test_parse_matches_reference(c):
    info = PP.parse(src(c))
    ref = c["reference"]
    assert info["name"] == ref["name"]
    got = [info["params"][k] for k in ARGS]
    got[-1] = info["ref_aa_shift"]  # writeToCircom passes extractFromDg15's byte offset (:795)
    assert [str(v) for v in got] == ref["circom_args"]
    assert info["params"]["aa_shift"] == 8 * info["ref_aa_shift"]


def _layout_ok(params):
    try:
        native.layout_witness_size(params)
        return True
    except native.PzkError:
        return False


@pytest.mark.parametrize("c", CASES, ids=lambda c: "sig%d_%d_%s" % (c["sig"], c["index"], "_".join(sorted(c["options"]))))
def test_rows_match_reference_json(c):
    ref = c["reference"]
    params = PP.parse(src(c))["params"]
    if not _layout_ok(params):
        pytest.skip("instance %s is outside the builder's parameter set" % (params,))
    j = ref["inputs"]
    ident = PP.identity_elements(int(j["slaveMerkleRoot"], 16), int(j["skIdentity"], 16))[None]
    rows, st = PP.input_rows(params, [src(c)], ident, threads=1)
    sizes_fit = len(j["signedAttributes"]) == 1024 and len(j["dg1"]) == 1024
    if not sizes_fit:  # e.g. SIG 13: the signed attributes pad to 2 x 1024 bits, the circuit takes 1024
        assert st[0] == 4 and not rows.any()
        return
    assert st[0] == 0, PP.PP_STATUS[int(st[0])]
    np.testing.assert_array_equal(rows[0], reference_row(ref, params, rows.shape[1]))


def test_bulk_threads_and_statuses():
    canon = next(c for c in CASES if c["sig"] == 1 and not c["options"])
    params = PP.parse(src(canon))["params"]
    bad = dict(src(canon), sod=base64.b64encode(base64.b64decode(canon["sod"])[:-40]).decode())
    batch = [src(canon)] * 37 + [bad] + [src(c) for c in CASES]
    rows1, st1 = PP.input_rows(params, batch, threads=1)
    rows8, st8 = PP.input_rows(params, batch, threads=8)
    np.testing.assert_array_equal(rows1, rows8)
    np.testing.assert_array_equal(st1, st8)
    assert (st1[:37] == 0).all() and st1[37] == 1
    for c, s in zip(CASES, st1[38:]):
        p = PP.parse(src(c))["params"]
        assert (s == 0) == (p == params), (c["sig"], c["options"], s)
        if p != params:
            assert s == (2 if p["sig"] == 0 else 3)  # getSigType 0 (UNKNOWN) before the parameter check
    assert not rows1[37].any()


def test_parse_errors_are_reported():
    canon = next(c for c in CASES if c["sig"] == 1 and not c["options"])
    with pytest.raises(native.PzkError, match="pzk_passport_parse"):
        PP.parse(dict(src(canon), sod=base64.b64encode(b"\x30\x03\x02\x01").decode()))
    with pytest.raises(native.PzkError):
        PP.parse(dict(src(canon), sod=""))


def test_ecdsa_p224_bp384_sods(oracle):
    """EF.SOD of ECDSA signers the reference classifies as SIGNATURE_TYPE 24 / 25 (process_passport.js getSigType by the
    key's curve parameter a). brainpoolP384r1 (SHA-384 throughout; signed attributes without signingTime, so they fit
    the circuit's one 1024-bit block): the rows verify in the CPU restatement (every check of the circuit passes on
    a signature made over real DER). secp224r1: processPassport's getChunkedParams (:590-626) cuts the key and the
    signature into 4 x 64-bit chunks where the circuit takes 7 x 32 (registerIdentityBuilder.circom:90-94), so no
    input the reference pipeline writes fits the SIG 24 circuit: status PZK_PP_LIMBS."""
    from pzkwit import sodgen
    pp = sodgen.make_passport(25, sodgen.signer_key(25), 0, signing_time=False)
    info = PP.parse(pp)
    assert info["params"]["sig"] == 25 and info["chunk_number"] == 6 and info["chunk_bits"] == 64
    rows, st = PP.input_rows(info["params"], [pp])
    assert st[0] == 0
    assert oracle.register_witness(oracle.register_params(**info["params"]), rows[0])[0] == 0
    pp = sodgen.make_passport(24, sodgen.signer_key(24), 0)
    info = PP.parse(pp)
    assert info["params"]["sig"] == 24 and (info["chunk_number"], info["chunk_bits"]) == (4, 64)
    _, st = PP.input_rows(info["params"], [pp])
    assert PP.PP_STATUS[int(st[0])] == "limbs"
