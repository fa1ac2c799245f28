"""Writes the circom-shaped signal maps (--O1 / --O2 approximations) of the benchmarked instances to
passport-zk-circuits_amd/data/shape/<name>_o<level>.npz (oracle/r1cs_shape.inc.c derives them from the restated
constraints; pzkwit/symmap.py load_shape reads them). A tool: it imports the test-infrastructure checker under
oracle/, the product path only reads the committed files.

    python tools/gen_shape_maps.py            # every map
    python tools/gen_shape_maps.py --check    # regenerate and compare with the committed files
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "passport-zk-circuits_amd"))

import pyr1cs  # noqa: E402
from pzkwit import inputs as I, native, symmap  # noqa: E402


def instances():
    """name -> (checker circuit, arg, checker params, pzk params, circuit id, size_arg)."""
    return {
        "register_canonical": ("register", 0, I.CANONICAL, I.CANONICAL, native.PZK_CIRCUIT_REGISTER, 0),
        "register_sig20": ("register", 0, I.instance_params(20), I.instance_params(20), native.PZK_CIRCUIT_REGISTER, 0),
        "query": ("query", 0, {}, {"doc": 0}, native.PZK_CIRCUIT_QUERY, 80),
    }


def make(name, level):
    circ, arg, ck_params, params, circuit, size_arg = instances()[name]
    if circuit == native.PZK_CIRCUIT_REGISTER:
        info = native.layout_info(params)
    else:
        info = native.layout_info(params, circuit, size_arg)
    n = int(info.witness_size)
    st = pyr1cs.structure(circ, n, arg=arg, **ck_params)
    try:
        wit, m = pyr1cs.shape_map(st, n, 1 + int(info.n_outputs) + int(info.n_inputs), level)
    finally:
        pyr1cs.free_structure(st)
    return wit, m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    os.makedirs(symmap.SHAPE_DIR, exist_ok=True)
    bad = 0
    for name in a.names or instances():
        for level in (1, 2):
            wit, m = make(name, level)
            path = symmap.shape_path(name, level)
            if a.check:
                same = os.path.exists(path) and np.array_equal(symmap.load_shape(name, level), wit)
                print("%-24s O%d %s" % (name, level, "ok" if same else "DIFFERS"))
                bad += not same
            else:
                symmap.save_shape(path, wit)
                print("%-24s O%d: %d of %d signals (%.3f) -> %s" % (name, level, m - 1, wit.shape[0] - 1,
                                                                    (m - 1) / (wit.shape[0] - 1), path))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
