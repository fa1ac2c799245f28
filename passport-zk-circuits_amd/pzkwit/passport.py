"""ctypes binding of the bulk SOD preprocessor (include/pzkpassport.h): passports as the reference's
processPassport reads them (test/process_passport.js:674-816; {dg1, dg15, sod} JSON, base64 or hex
fields) -> RegisterIdentityBuilder parameters and flat input rows for pzk_witness_batch.
Host only: no device is touched."""
import base64
import ctypes
import re

import numpy as np

from . import native

PP_STATUS = {0: "OK", 1: "parse", 2: "unknown signature / AA curve", 3: "other instance parameters",
             4: "padded length", 5: "limbs"}
_HEX = re.compile(r"^\s*(?:[0-9A-Fa-f][0-9A-Fa-f]\s*)+$")  # reHex (process_passport.js:6)


class PassportSrc(ctypes.Structure):
    _fields_ = [("dg1", ctypes.c_void_p), ("dg1_len", ctypes.c_size_t), ("dg15", ctypes.c_void_p),
                ("dg15_len", ctypes.c_size_t), ("sod", ctypes.c_void_p), ("sod_len", ctypes.c_size_t)]


class PassportInfo(ctypes.Structure):
    _fields_ = [("params", native.PzkParams)] + [(n, ctypes.c_int32) for n in (
        "ref_aa_shift", "dg_hash_bytes", "hash_bytes", "dg1_len", "dg15_len", "ec_len", "sa_len", "chunk_number",
        "chunk_bits", "salt", "reserved")] + [("name", ctypes.c_char * 128)]


def _lib():
    L = native.lib()
    if not getattr(L, "_pp_ready", False):
        L.pzk_passport_parse.argtypes = [ctypes.POINTER(PassportSrc), ctypes.POINTER(PassportInfo)]
        L.pzk_passport_inputs.argtypes = [ctypes.POINTER(native.PzkParams), ctypes.POINTER(PassportSrc), ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L._pp_ready = True
    return L


def field_bytes(v):
    """A passport JSON field -> bytes: processPassport's reHex test, else base64 (:676-685)."""
    if v is None or v == "":
        return b""
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    return bytes.fromhex("".join(v.split())) if _HEX.match(v) else base64.b64decode(v)


class Sources:
    """Passports marshalled once into a pzk_passport_src array (byte buffers kept alive)."""

    def __init__(self, arr, keep, n):
        self.arr, self.keep, self.n = arr, keep, n

    def __len__(self):
        return self.n


def sources(passports):
    return passports if isinstance(passports, Sources) else Sources(*_srcs(passports), len(passports))


def _srcs(passports):
    keep, arr = [], (PassportSrc * max(1, len(passports)))()
    for i, p in enumerate(passports):
        parts = []
        for f in ("dg1", "dg15", "sod"):
            b = field_bytes(p.get(f))
            buf = ctypes.create_string_buffer(b, len(b)) if b else None
            keep.append(buf)
            parts += [ctypes.cast(buf, ctypes.c_void_p) if buf is not None else None, len(b)]
        arr[i] = PassportSrc(*parts)
    return arr, keep


_SHORT = {v: k for k, v in native._PARAM_MAP.items()}


def parse(passport):
    """One passport -> dict: params (short names, inputs.CANONICAL style; shifts in bits), the reference's
    name and AA_SHIFT argument, digest sizes, chunking."""
    arr, _keep = _srcs([passport])
    info = PassportInfo()
    native._check(_lib().pzk_passport_parse(arr, ctypes.byref(info)))
    params = {_SHORT[n]: getattr(info.params, n) for n, _ in native.PzkParams._fields_ if n in _SHORT}
    out = {n: getattr(info, n) for n, _ in PassportInfo._fields_ if n not in ("params", "name", "reserved")}
    out.update(params=params, name=info.name.decode())
    return out


def input_rows(params, passports, identity=None, threads=0, out=None):
    """Bulk: passports -> (rows (n, n_inputs, 32) uint8, status (n,) int32). identity: (n, 82, 32) uint8
    field elements (slaveMerkleRoot, skIdentity, 80 branches) or None for zeros; out: a rows array to reuse
    (e.g. pinned host memory)."""
    p = native.PzkParams(circuit=native.PZK_CIRCUIT_REGISTER)
    for k, v in native.param_fields(params).items():
        setattr(p, k, v)
    info = native.PzkInfo()
    native._check(native.lib().pzk_layout_query(ctypes.byref(p), ctypes.byref(info), None))
    n = len(passports)
    rows = out if out is not None else np.zeros((n, int(info.n_inputs), 32), dtype=np.uint8)
    assert rows.shape == (n, int(info.n_inputs), 32) and rows.dtype == np.uint8 and rows.flags.c_contiguous
    status = np.zeros(n, dtype=np.int32)
    ident = None
    if identity is not None:
        ident = np.ascontiguousarray(identity, dtype=np.uint8)
        assert ident.shape == (n, 82, 32), ident.shape
    src = sources(passports)
    native._check(_lib().pzk_passport_inputs(ctypes.byref(p), src.arr, n,
                                             ident.ctypes.data if ident is not None else None,
                                             rows.ctypes.data, status.ctypes.data, int(threads)))
    return rows, status


def identity_elements(root, sk, branches=None):
    """(slaveMerkleRoot, skIdentity, branches) ints -> (82, 32) uint8 little-endian field elements."""
    from .field import P
    vals = [root, sk] + list(branches or [0] * 80)
    return np.stack([np.frombuffer(int(v % P).to_bytes(32, "little"), dtype=np.uint8) for v in vals])
