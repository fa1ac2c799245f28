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
def test_js_addon_cpu():
    """addon loads and exports; input marshalling and error texts; no CPU fallback without a GPU."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")  # the no-device path even where a GPU exists
    r = subprocess.run(["node", "test_witness_calculator.js", "cpu"], cwd=JS, capture_output=True, text=True,
                       timeout=120, env=env)
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
    r = subprocess.run(["node", "test_witness_calculator.js", "gpu", str(inp), str(out)], cwd=JS,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    data = out.read_bytes()
    prm = oracle.register_params(**I.CANONICAL)
    rc, ref = oracle.register_witness(prm, I.pack_register_inputs(pp))
    assert rc == 0
    assert data[:4] == b"wtns" and len(data) == 76 + ref.size
    got = np.frombuffer(data[76:], dtype=np.uint8).reshape(ref.shape)
    assert (got == ref).all()
