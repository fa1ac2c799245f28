"""Generate tests/golden/sod_vectors.json: synthetic passports with real EF.SOD files (pzkwit.sodgen),
run through the reference's own processPassport by tools/gen_sod_fixtures.js on this container's
Node 12. Runs here only (the reference is not on the GPU box):
    python tools/gen_sod_fixtures.py /root/reference/test
The fixture holds each passport's files (base64) and what the reference wrote for it.
"""
import base64
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "passport-zk-circuits_amd"))

from pzkwit import sodgen  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "sod_vectors.json")

# (SIGNATURE_TYPE, passport index, make_passport options): the canonical layout (five DGs, DG15 last),
# other DG counts / no DG15 / no signingTime (other shifts and block counts), TD1, every scheme
CASES = [
    (1, 0, {}), (1, 1, {"n_dgs": 4}), (1, 2, {"dg15": False, "n_dgs": 3}), (1, 3, {"signing_time": False}),
    (1, 4, {"td1": True}), (1, 5, {"dg_hash": 224}), (3, 0, {}), (10, 0, {}), (11, 0, {}), (12, 0, {}),
    (13, 0, {"n_dgs": 3}), (20, 0, {}), (21, 0, {}), (20, 1, {"dg15": False}),
    # quirk paths: a key named by OID (P-256: getSigType 0; secp521r1: SIG 27, 66-bit chunks), PSS parameters
    # without saltLength (the salt reads "(2 elem)": SIG 0), a digest found at an odd hex digit, RSA-4096 / 3072
    (20, 2, {"named_curve": "prime256v1"}), (27, 0, {"named_curve": "secp521r1"}), (11, 1, {"pss_salt_param": False}),
    (1, 6, {"odd_dg1": True}), (2, 0, {}), (14, 0, {}),
]


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/test"
    keys = {}
    cases = []
    with tempfile.TemporaryDirectory() as tmp:
        for k, (sig, idx, opt) in enumerate(CASES):
            if sig not in keys:
                keys[sig] = sodgen.signer_key(sig)
            pp = sodgen.make_passport(sig, keys[sig], idx, **opt)
            files = {f: base64.b64encode(pp[f]).decode() for f in ("dg1", "dg15", "sod")}
            fname = "case%02d.json" % k
            with open(os.path.join(tmp, fname), "w") as fh:
                json.dump(files, fh)
            cases.append(dict(file=fname, sig=sig, index=idx, options=opt, **files))
        out = os.path.join(tmp, "out.json")
        subprocess.check_call(["node", "--harmony-optional-chaining", "--harmony-private-methods",
                               os.path.join(REPO, "tools", "gen_sod_fixtures.js"), ref, tmp, out])
        with open(out) as fh:
            res = json.load(fh)
    by_file = {c["file"]: c for c in res["cases"]}
    for c in cases:
        c["reference"] = by_file[c["file"]]
    with open(OUT, "w") as fh:
        json.dump({"source": res["source"] + " (tools/gen_sod_fixtures.js)", "cases": cases}, fh, indent=0)
    print("wrote", OUT, len(cases), "cases")


if __name__ == "__main__":
    main()
