"""The Node host layer (passport-zk-circuits_amd/js): the N-API addon over the C-ABI and the
witness_calculator.js mirror of circom's calculator API."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from pzkwit import inputs as I

JS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "passport-zk-circuits_amd", "js")
ADDON = os.path.join(JS, "build", "pzkwit.node")

needs_node = pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(ADDON),
                                reason="node or the built addon (make -C passport-zk-circuits_amd/js) missing")


@needs_node
def test_js_addon_cpu(tmp_path):
    """addon loads and exports; input marshalling and error texts; no CPU fallback without a GPU; the
    bulk SOD preprocessor binding (passportParse / passportInputs) gives the reference-checked circuit names
    (tests/golden/sod_vectors.json) and the same rows and statuses as the C-ABI called from Python."""
    from pzkwit import passport as PP
    cases = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sod_vectors.json")))["cases"]
    params = PP.parse(cases[0])["params"]
    rows, st = PP.input_rows(params, cases, threads=2)
    (tmp_path / "rows.bin").write_bytes(rows.tobytes())
    jp = {"circuit": 0, "SIGNATURE_TYPE": params["sig"], "DG_HASH_TYPE": params["dg_hash"],
          "DOCUMENT_TYPE": params["doc"], "EC_BLOCK_NUMBER": params["ec_blocks"], "EC_SHIFT": params["ec_shift"],
          "DG1_SHIFT": params["dg1_shift"], "AA_SIGNATURE_ALGO": params["aa"], "DG15_SHIFT": params["dg15_shift"],
          "DG15_BLOCK_NUMBER": params["dg15_blocks"], "AA_SHIFT": params["aa_shift"]}
    pp = {"params": jp, "status": [int(x) for x in st], "names": [c["reference"]["name"] for c in cases],
          "passports": [{f: c[f] or None for f in ("dg1", "dg15", "sod")} for c in cases]}
    (tmp_path / "pp.json").write_text(json.dumps(pp))
    assert (st == 0).any() and (st != 0).any()  # both paths of the binding are exercised
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")  # the no-device path even where a GPU exists
    r = subprocess.run(["node", "test_witness_calculator.js", "cpu", str(tmp_path / "pp.json"), str(tmp_path / "rows.bin")],
                       cwd=JS, capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr


@needs_node
@pytest.mark.gpu
def test_js_register_wtns_matches_oracle(oracle, tmp_path):
    """calculateWTNSBin through node on the reference's JSON input format == oracle witness + header."""
    gen = I.PassportGen(seed=3, n_keys=2)
    pp = gen.passport_at(7, smt_depth=5)
    inp = tmp_path / "input.json"
    inp.write_text(json.dumps(I.passport_json(pp)))
    out = tmp_path / "out.wtns"
    # three different passports for the concurrency check, and a .sym map (with merged witness indices)
    from pzkwit import native, symmap
    extra = tmp_path / "extra.json"
    n_o0 = native.layout_witness_size(I.CANONICAL)
    keep = symmap.synthetic_keep(n_o0, 1 + 4 + 5778, fraction=4)
    merged = symmap.synthetic_keep(n_o0, 0, fraction=5, salt=0x33)
    three = [gen.passport_at(k, smt_depth=d) for k, d in ((8, 3), (9, 0), (10, 7))]
    extra.write_text(json.dumps({"inputs": [I.passport_json(p) for p in three],
                                 "sym": symmap.sym_text(keep, merged=merged)}))
    outdir = tmp_path / "wtns"
    outdir.mkdir()
    r = subprocess.run(["node", "--expose-gc", "test_witness_calculator.js", "gpu", str(inp), str(out), str(extra),
                        str(outdir)], cwd=JS, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "js stream ok" in r.stdout, r.stdout
    data = out.read_bytes()
    prm = oracle.register_params(**I.CANONICAL)
    rc, ref = oracle.register_witness(prm, I.pack_register_inputs(pp))
    assert rc == 0
    assert data[:4] == b"wtns" and len(data) == 76 + ref.size
    got = np.frombuffer(data[76:], dtype=np.uint8).reshape(ref.shape)
    assert (got == ref).all()
    # writeWTNSFiles (streamed, one .wtns per input as gen-witness.sh:25): each file == header + oracle witness
    for i, p in enumerate([pp] + three):
        f = (outdir / ("w%d.wtns" % i)).read_bytes()
        rc, ref = oracle.register_witness(prm, I.pack_register_inputs(p))
        assert rc == 0 and f[:76] == data[:76] and f[76:] == ref.tobytes(), i
