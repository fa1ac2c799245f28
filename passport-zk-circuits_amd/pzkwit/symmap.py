"""Signal -> witness maps in circom's .sym format (pzk_instance_create_mapped, include/pzkwit.h).

circom --sym writes one line per signal: "signal_idx,witness_idx,component_idx,name", witness_idx
-1 for a signal its --O1/--O2 simplification eliminated (circuits/scripts/compile-circuit.sh:34). The
witness the prover reads (circuits/scripts/prove.sh:27) is then element k = the signal whose
witness_idx is k. Here the signal indices are the --O0 numbering of DESIGN.md §2; a real circom .sym
can be dropped in where circom is available (none is here: SURVEY.md §8c).
"""
import numpy as np


def sym_text(keep, names=None, merged=None):
    """keep: bool array over the O0 signals (index 0 = the constant 1, ignored). Kept signals get
    witness indices 1, 2, ... in O0 order. merged: optional bool array; a merged signal that is not kept
    shares the witness index of the closest kept signal before it (circom's simplification maps equal
    signals onto one witness index; snarkjs loadSymbols joins their names with '|')."""
    keep = np.asarray(keep, dtype=bool)
    wit = np.full(keep.shape[0], -1, dtype=np.int64)
    idx = np.flatnonzero(keep[1:]) + 1
    wit[idx] = np.arange(1, idx.size + 1)
    if merged is not None:
        last = np.maximum.accumulate(np.where(keep, np.arange(keep.shape[0]), 0))
        m = np.asarray(merged, dtype=bool) & ~keep & (last > 0)
        wit[m] = wit[last[m]]
    lines = ["%d,%d,0,%s" % (s, wit[s], names[s] if names else "s%d" % s) for s in range(1, keep.shape[0])]
    return "\n".join(lines) + "\n"


def parse_sym(text):
    """-> inv: inv[k] = O0 signal index of output element k (inv[0] = 0)."""
    pairs = {}
    for ln in text.splitlines():
        if not ln.strip():
            continue
        sig, wit = (int(x) for x in ln.split(",")[:2])
        if wit >= 0:  # several signals on one index: the lowest signal index stands for them (runtime.cpp parse_sym)
            pairs[wit] = min(sig, pairs.get(wit, sig))
    n = max(pairs) + 1
    inv = np.zeros(n, dtype=np.int64)
    for k in range(1, n):
        inv[k] = pairs[k]
    return inv


def synthetic_keep(o0_size, n_prefix, fraction=4, salt=0x5A):
    """A deterministic synthetic map (NOT circom's O2): the outputs and inputs (the first n_prefix
    signals) plus every signal whose index hashes to 0 mod `fraction`."""
    s = np.arange(o0_size, dtype=np.uint64)
    h = (s * np.uint64(0x9E3779B97F4A7C15) + np.uint64(salt)) >> np.uint64(40)
    keep = (h % np.uint64(fraction)) == 0
    keep[:n_prefix] = True
    return keep


# ---- circom-shaped maps (approximate --O1 / --O2; tools/gen_shape_maps.py, oracle/r1cs_shape.inc.c)
import os  # noqa: E402

SHAPE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "shape")


def shape_path(name, level):
    return os.path.join(SHAPE_DIR, "%s_o%d.npz" % (name, level))


def save_shape(path, wit):
    """wit: witness index per O0 signal (-1 = removed), stored as differences (the map is mostly a ramp)."""
    d = np.diff(np.asarray(wit, dtype=np.int64), prepend=0).astype(np.int32)
    np.savez_compressed(path, dwit=d)


def load_shape(name, level):
    """-> wit (int32 per O0 signal): the --O<level>-shaped map of a committed instance. The maps follow circom's
    documented simplification rules applied to the restated constraints; which signals circom itself keeps is
    parity unpinned."""
    with np.load(shape_path(name, level)) as z:
        return np.cumsum(z["dwit"].astype(np.int64)).astype(np.int32)


def sym_text_wit(wit, names=None):
    """circom .sym text of a witness-index array (signal 0, the constant, is not listed)."""
    wit = np.asarray(wit)
    s = np.arange(1, wit.shape[0])
    if names is None:
        lines = np.char.add(np.char.add(np.char.add(s.astype(str), ","), wit[1:].astype(str)), ",0,s")
        lines = np.char.add(lines, s.astype(str))
    else:
        lines = ["%d,%d,0,%s" % (i, wit[i], names[i]) for i in s]
    return "\n".join(lines) + "\n"
