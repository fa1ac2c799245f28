"""Generate tests/golden/process_passport_vectors.json: raw synthetic passports (pzkwit.inputs.PassportGen)
and edge-case messages, run through the reference's own input functions by tools/gen_input_fixtures.js
on this container's Node 12. Runs here only (the reference is not on the GPU box):
    python tools/gen_input_fixtures.py /root/reference/test
"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "passport-zk-circuits_amd"))

from pzkwit import inputs as I  # noqa: E402
from pzkwit.field import SplitMix64  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "process_passport_vectors.json")


def hx(b):
    return b.hex()


def passport_case(sig, i, seed):
    """One synthetic passport of SIGNATURE_TYPE sig, as the raw fields processPassport extracts."""
    params = I.instance_params(sig)
    g = I.PassportGen(seed=seed, n_keys=2, params=params, workers=1)
    pp = g.passport_at(i)
    key = g.keys[i % len(g.keys)]
    if isinstance(key, I.EcKey):
        curve = "brainpoolP256r1" if sig == 21 else "secp256r1"
        pk = {"x": "%064x" % key.q[0], "y": "%064x" % key.q[1], "param": curve}
        sigd = {"r": "%064x" % pp["sig"][0], "s": "%064x" % pp["sig"][1]}
    else:
        nbytes = (key.n.bit_length() + 7) // 8
        pk = {"n": "%0*x" % (2 * nbytes, key.n)}
        sigd = {"n": "%0*x" % (2 * nbytes, pp["sig"])}
        if 10 <= sig <= 14:
            sigd["salt"] = I.pss_salt_len(sig)
    return {"name": "sig%d_passport%d" % (sig, i), "sig_type": sig, "index": i, "seed": seed,
            "passport": {"dg1": hx(pp["dg1"]), "dg15": hx(pp["dg15"]), "ec": hx(pp["ec"]), "sa": hx(pp["sa"]),
                         "pk": pk, "sig": sigd}}


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/test"
    rng = SplitMix64(0x77)
    cases = []
    for sig, n in ((1, 3), (2, 1), (3, 1), (11, 1), (10, 1), (20, 2), (21, 1)):
        for i in range(n):
            cases.append(passport_case(sig, i, 0x700 + sig))
    # padding edge cases: lengths around the block boundaries, both block sizes, leading zero bytes
    pads = []
    for L in (0, 1, 55, 56, 57, 63, 64, 65, 111, 112, 119, 120, 127, 128, 200):
        pads.append([rng.bytes(L).hex(), 512])
        pads.append([rng.bytes(L).hex(), 1024])
    pads.append([("00" * 3) + rng.bytes(40).hex(), 512])   # leading zero bytes inside the first block
    pads.append([("00" * 70) + rng.bytes(10).hex(), 512])  # a whole zero first block (the BigInt round trip drops it)
    limbs = []
    for n, k in ((64, 32), (64, 64), (64, 48), (64, 15), (64, 4), (66, 8)):
        for _ in range(3):
            limbs.append([n, k, str(rng.below(1 << min(n * k, 4096)))])
    limbs.append([64, 32, str((1 << 2048) - 1)])
    hashes = [[ln, rng.bytes(L).hex()] for ln in (20, 28, 32, 48, 64) for L in (0, 64, 200)]
    cases.append({"name": "edges", "padding": pads, "limbs": limbs, "hash": hashes})
    with tempfile.TemporaryDirectory() as td:
        cin = os.path.join(td, "cases.json")
        json.dump(cases, open(cin, "w"))
        subprocess.check_call(["node", os.path.join(REPO, "tools", "gen_input_fixtures.js"), ref, cin, OUT])
    print("fixture:", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
