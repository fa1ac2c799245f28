"""ctypes front-end of the CPU oracle (oracle/witness_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker. The product path
(passport-zk-circuits_amd/) never imports anything under oracle/.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB = os.path.join(HERE, "build", "liboracle.so")
POSEIDON_BIN = os.path.join(REPO, "passport-zk-circuits_amd", "data", "poseidon_t2_6.bin")
# generator tables by curve index (SIGNATURE_TYPE 20, 21, 24, 25)
EC_TABLES = [os.path.join(REPO, "passport-zk-circuits_amd", "data", n) for n in
             ("p256_gpow8.bin", "bp256_gpow8.bin", "p224_gpow8.bin", "bp384_gpow8.bin")]
P256_BIN, BP256_BIN = EC_TABLES[0], EC_TABLES[1]

P = 21888242871839275222246405745257275088548364400416034343698204186575808495617


class OrcParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "sig", "dg_hash", "doc", "ec_blocks", "ec_shift", "dg1_shift", "aa",
        "dg15_shift", "dg15_blocks", "aa_shift")]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.orc_load_poseidon.argtypes = [ctypes.c_char_p]
        L.orc_register_witness_size.restype = ctypes.c_size_t
        L.orc_register_witness_size.argtypes = [ctypes.POINTER(OrcParams)]
        L.orc_register_n_inputs.restype = ctypes.c_size_t
        L.orc_register_n_inputs.argtypes = [ctypes.POINTER(OrcParams)]
        L.orc_register_witness.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_void_p, ctypes.c_void_p]
        L.orc_poseidon_witness_size.restype = ctypes.c_size_t
        L.orc_poseidon_witness.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_poseidon_hash.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_sha256_witness_size.restype = ctypes.c_size_t
        L.orc_sha256_witness.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_sha1_witness_size.restype = ctypes.c_size_t
        L.orc_sha1_witness.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_sha512_witness_size.restype = ctypes.c_size_t
        L.orc_sha512_witness_size.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_sha512_witness.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_query_witness_size.restype = ctypes.c_size_t
        L.orc_query_witness_size.argtypes = [ctypes.c_int]
        L.orc_query_n_inputs.restype = ctypes.c_size_t
        L.orc_query_n_inputs.argtypes = [ctypes.c_int]
        L.orc_query_witness.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        rc = L.orc_load_poseidon(POSEIDON_BIN.encode())
        if rc != 0:
            raise RuntimeError("oracle: cannot load Poseidon constants (%d)" % rc)
        L.orc_load_ec_table.argtypes = [ctypes.c_int, ctypes.c_char_p]
        for curve, path in enumerate(EC_TABLES):
            rc = L.orc_load_ec_table(curve, path.encode())
            if rc != 0:
                raise RuntimeError("oracle: cannot load the generator table %s (%d)" % (path, rc))
        _lib = L
    return _lib


def to_elems(ints):
    """python ints (already reduced < p) -> (n,32) uint8 little-endian."""
    out = np.zeros((len(ints), 32), dtype=np.uint8)
    for i, v in enumerate(ints):
        out[i] = np.frombuffer(int(v).to_bytes(32, "little"), dtype=np.uint8)
    return out


def from_elem(b):
    return int.from_bytes(bytes(b), "little")


def poseidon(ins):
    L = lib()
    arr = to_elems([x % P for x in ins])
    out = np.zeros(32, dtype=np.uint8)
    L.orc_poseidon_hash(len(ins), arr.ctypes.data, out.ctypes.data)
    return from_elem(out)


def poseidon_witness(ins):
    L = lib()
    n = len(ins)
    sz = L.orc_poseidon_witness_size(n)
    w = np.zeros((sz, 32), dtype=np.uint8)
    arr = to_elems([x % P for x in ins])
    rc = L.orc_poseidon_witness(n, arr.ctypes.data, w.ctypes.data)
    return rc, w


def sha256_witness(in_elems, blocks):
    """in_elems: (512*blocks, 32) uint8 array of input signals."""
    L = lib()
    sz = L.orc_sha256_witness_size(blocks)
    w = np.zeros((sz, 32), dtype=np.uint8)
    a = np.ascontiguousarray(in_elems, dtype=np.uint8)
    rc = L.orc_sha256_witness(blocks, a.ctypes.data, w.ctypes.data)
    return rc, w


def register_params(**kw):
    return OrcParams(**kw)


def register_sizes(params):
    L = lib()
    return L.orc_register_n_inputs(ctypes.byref(params)), L.orc_register_witness_size(ctypes.byref(params))


def register_witness(params, inputs, out=None):
    """inputs: (nIn,32) uint8 in witness order. Returns (rc, witness (nWit,32) uint8)."""
    L = lib()
    nin, nw = register_sizes(params)
    a = np.ascontiguousarray(inputs, dtype=np.uint8)
    assert a.shape == (nin, 32), (a.shape, nin)
    w = out if out is not None else np.zeros((nw, 32), dtype=np.uint8)
    rc = L.orc_register_witness(ctypes.byref(params), a.ctypes.data, w.ctypes.data)
    return rc, w


def sha1_witness(in_elems, blocks):
    """Sha1HashChunks(blocks) witness; in_elems: (512*blocks, 32) uint8 array of input signals."""
    L = lib()
    sz = L.orc_sha1_witness_size(blocks)
    w = np.zeros((sz, 32), dtype=np.uint8)
    a = np.ascontiguousarray(in_elems, dtype=np.uint8)
    rc = L.orc_sha1_witness(blocks, a.ctypes.data, w.ctypes.data)
    return rc, w


def sha512_witness(in_elems, blocks, out_bits=512):
    """Sha512HashChunks(blocks) (out_bits 512) / Sha384HashChunks(blocks) (384) witness;
    in_elems: (1024*blocks, 32) uint8 array of input signals."""
    L = lib()
    sz = L.orc_sha512_witness_size(blocks, out_bits)
    w = np.zeros((sz, 32), dtype=np.uint8)
    a = np.ascontiguousarray(in_elems, dtype=np.uint8)
    rc = L.orc_sha512_witness(blocks, out_bits, a.ctypes.data, w.ctypes.data)
    return rc, w


def query_sizes(td1=False):
    """QueryIdentity(80) (td1: QueryIdentityTD1): (inputs, witness elements)."""
    L = lib()
    return L.orc_query_n_inputs(int(td1)), L.orc_query_witness_size(int(td1))


def query_witness(inputs, out=None, td1=False):
    """QueryIdentity(80) witness; inputs (842 | 858, 32) uint8 in declaration order. Returns (rc, (nWit, 32) uint8)."""
    L = lib()
    nin, nw = query_sizes(td1)
    a = np.ascontiguousarray(inputs, dtype=np.uint8)
    assert a.shape == (nin, 32), (a.shape, nin)
    w = out if out is not None else np.zeros((nw, 32), dtype=np.uint8)
    rc = L.orc_query_witness(int(td1), a.ctypes.data, w.ctypes.data)
    return rc, w
