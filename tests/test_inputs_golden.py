"""CPU: the caller-side input formats (pzkwit/inputs.py) against the reference's own
input-preparation functions. tests/golden/process_passport_vectors.json holds outputs of
test/process_passport.js's padding / computeHash / bigintToArray / bigintToArrayString /
getChunkedParams / getFakeIdenData (and test/poseidon.js inside getFakeIdenData), run on Node 12 in
the build container by tools/gen_input_fixtures.{py,js} over raw synthetic passports and edge cases."""
import hashlib
import json
import os

import numpy as np
import pytest

from pzkwit import inputs as I, witness_calculator as WC
from pzkwit.field import P

GOLD = os.path.join(os.path.dirname(__file__), "golden", "process_passport_vectors.json")
D = json.load(open(GOLD))
EDGES = next(c for c in D["cases"] if c["name"] == "edges")
PASSPORTS = [c for c in D["cases"] if "passport" in c]


def _bits(s):
    return "".join(str(int(b)) for b in s)


@pytest.mark.parametrize("k", range(len(EDGES["padding"])))
def test_padding_matches_reference(k):
    """padding() :11-91 (both block sizes) and processPassport's bit-array round trip :701-757,
    including the whole-zero-first-block case where BigInt(...).toString(2) drops a block."""
    c = EDGES["padding"][k]
    msg = bytes.fromhex(c["hex"])
    assert I.sha_pad(msg, c["block_bits"]).hex() == c["padded"]
    assert _bits(I.padded_bits(msg, c["block_bits"])) == c["bits"]


def test_limbs_match_reference():
    """bigintToArray / bigintToArrayString :113-135 (limb size, count, overflow truncation)."""
    for c in EDGES["limbs"]:
        got = I.chunk_limbs(int(c["x"]), c["n"], c["k"])
        assert [str(v) for v in got] == c["array"] == c["array_string"]


def test_hashes_match_reference():
    """computeHash :93-111 output lengths 20/28/32/48/64 -> SHA-1/224/256/384/512."""
    algo = {20: hashlib.sha1, 28: hashlib.sha224, 32: hashlib.sha256, 48: hashlib.sha384, 64: hashlib.sha512}
    for c in EDGES["hash"]:
        assert algo[c["len"]](bytes.fromhex(c["hex"])).hexdigest() == c["digest"]


@pytest.mark.parametrize("case", PASSPORTS, ids=[c["name"] for c in PASSPORTS])
def test_passport_json_matches_reference(case):
    """The whole input JSON of a synthetic passport — padded DG1/DG15/EC/SA bit arrays, pubkey and
    signature limbs (getChunkedParams :590-626), skIdentity and slaveMerkleRoot (getFakeIdenData
    :628-657, Poseidon from test/poseidon.js) — equals what the reference's functions make of the
    same raw bytes; and the marshalled JSON equals the packed input row the bench feeds the GPU."""
    sig, i, seed = case["sig_type"], case["index"], case["seed"]
    params = I.instance_params(sig)
    g = I.PassportGen(seed=seed, n_keys=2, params=params, workers=1)
    pp = g.passport_at(i)
    raw = case["passport"]["raw"]
    assert pp["dg1"].hex() == raw["dg1"] and pp["ec"].hex() == raw["ec"] and pp["sa"].hex() == raw["sa"]
    ref = case["passport"]["json"]
    js = I.passport_json(pp, params)
    for k in ("dg1", "dg15", "signedAttributes", "encapsulatedContent"):
        assert "".join(js[k]) == ref[k], k
    for k in ("pubkey", "signature", "skIdentity", "slaveMerkleRoot", "slaveMerkleInclusionBranches"):
        assert js[k] == ref[k], k
    assert case["passport"]["chunk_number"] == I.sig_input_len(sig)  # ECDSA: 4 limbs of x + 4 of y
    # JSON (the reference's format) -> flat rows == the packed rows of pack_register_inputs
    groups = [("slaveMerkleRoot", 1), ("encapsulatedContent", params["ec_blocks"] * 512), ("dg1", 1024),
              ("dg15", params["dg15_blocks"] * 512), ("signedAttributes", 1024),
              ("signature", I.sig_input_len(sig)), ("pubkey", I.sig_input_len(sig)),
              ("slaveMerkleInclusionBranches", 80), ("skIdentity", 1)]
    offs, o = [], 0
    for name, ln in groups:
        offs.append((name, o, ln))
        o += ln
    ref_json = dict(ref)
    for k in ("dg1", "dg15", "signedAttributes", "encapsulatedContent"):
        ref_json[k] = list(ref[k])
    buf = WC.marshal_inputs(offs, o, ref_json)
    assert (buf == I.pack_register_inputs(pp, params)).all()
    assert int(ref["skIdentity"], 16) < P
