"""ctypes front-end of the constraint checker (oracle/r1cs_check.c).

TEST INFRASTRUCTURE ONLY — imported by tests/ as a checker; the product path never imports
anything under oracle/."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libr1cs.so")


class Report(ctypes.Structure):
    _fields_ = [("n_constraints", ctypes.c_uint64), ("n_failed", ctypes.c_uint64),
                ("n_uncovered", ctypes.c_uint64), ("size_walked", ctypes.c_uint64),
                ("first_failed", ctypes.c_int64), ("first_line", ctypes.c_int32), ("oob", ctypes.c_int32),
                ("first_template", ctypes.c_char * 96), ("first_component", ctypes.c_uint64),
                ("first_uncovered", ctypes.c_int64), ("n_uncovered_nonzero", ctypes.c_uint64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["first_template"] = self.first_template.decode()
        return d


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(LIB)
        for fn in ("ck_sha256", "ck_sha1", "ck_poseidon_circuit"):
            getattr(L, fn).argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(Report)]
        L.ck_sha512.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(Report)]
        L.ck_load_poseidon.argtypes = [ctypes.c_char_p]
        L.ck_load_ec_table.argtypes = [ctypes.c_int, ctypes.c_char_p]
        L.ck_register.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(Report)]
        L.ck_query.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(Report)]
        _lib = L
    return _lib


def _run(fn, arg, wit):
    import numpy as np
    w = np.ascontiguousarray(wit, dtype=np.uint8)
    r = Report()
    rc = getattr(lib(), fn)(arg, w.ctypes.data, w.shape[0], ctypes.byref(r))
    return rc, r.as_dict()


def check_sha1(wit, blocks):
    """Sha1HashChunks(blocks) as main."""
    return _run("ck_sha1", blocks, wit)


def check_sha512(wit, blocks, out_bits=512):
    """Sha384HashChunks / Sha512HashChunks(blocks) as main."""
    import numpy as np
    w = np.ascontiguousarray(wit, dtype=np.uint8)
    r = Report()
    rc = lib().ck_sha512(blocks, out_bits, w.ctypes.data, w.shape[0], ctypes.byref(r))
    return rc, r.as_dict()


def check_sha256(wit, blocks):
    """Sha256HashChunks(blocks) as main: (rc, report); rc 0 = every constraint holds and the walk
    covered exactly the witness."""
    return _run("ck_sha256", blocks, wit)


class CkParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "sig", "dg_hash", "doc", "ec_blocks", "ec_shift", "dg1_shift", "aa",
        "dg15_shift", "dg15_blocks", "aa_shift")]


_pos_loaded = False


def _load_poseidon():
    global _pos_loaded
    if not _pos_loaded:
        path = os.path.join(os.path.dirname(HERE), "passport-zk-circuits_amd", "data", "poseidon_t2_6.bin")
        rc = lib().ck_load_poseidon(path.encode())
        if rc:
            raise RuntimeError("r1cs_check: cannot load Poseidon constants (%d)" % rc)
        data = os.path.join(os.path.dirname(HERE), "passport-zk-circuits_amd", "data")
        for curve, name in enumerate(("p256_gpow8.bin", "bp256_gpow8.bin", "p224_gpow8.bin", "bp384_gpow8.bin")):
            rc = lib().ck_load_ec_table(curve, os.path.join(data, name).encode())
            if rc:
                raise RuntimeError("r1cs_check: cannot load %s (%d)" % (name, rc))
        _pos_loaded = True


def check_poseidon(wit, n):
    """PoseidonHash(n) as main."""
    _load_poseidon()
    return _run("ck_poseidon_circuit", n, wit)


def check_register(wit, **params):
    """RegisterIdentityBuilder(...) as main (short parameter names of pzkwit.inputs.CANONICAL)."""
    import numpy as np
    _load_poseidon()
    p = CkParams(**params)
    w = np.ascontiguousarray(wit, dtype=np.uint8)
    r = Report()
    rc = lib().ck_register(ctypes.byref(p), w.ctypes.data, w.shape[0], ctypes.byref(r))
    return rc, r.as_dict()


def check_query(wit, td1=False):
    """QueryIdentity(80) witness (oracle/r1cs_query.inc.c; td1: QueryIdentityTD1) -> (rc, report dict)."""
    import numpy as np
    _load_poseidon()
    w = np.ascontiguousarray(wit, dtype=np.uint8)
    r = Report()
    rc = lib().ck_query(int(td1), w.ctypes.data, w.shape[0], ctypes.byref(r))
    return rc, r.as_dict()


class CkStruct(ctypes.Structure):
    _fields_ = [("n_cons", ctypes.c_uint64), ("n_sup", ctypes.c_uint64), ("cls", ctypes.POINTER(ctypes.c_uint8)),
                ("off", ctypes.POINTER(ctypes.c_uint64)), ("sup", ctypes.POINTER(ctypes.c_uint32))]


CIRCUITS = {"register": 0, "query": 1, "sha256": 2, "poseidon": 3}
QUAD, LIN, COPY, CONST = 0, 1, 2, 3


def _shape_lib():
    L = lib()
    if not getattr(L, "_shape_ready", False):
        L.ck_structure.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                                   ctypes.POINTER(CkStruct)]
        L.ck_struct_free.argtypes = [ctypes.POINTER(CkStruct)]
        L.ck_shape_map.argtypes = [ctypes.POINTER(CkStruct), ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
        L.ck_shape_map.restype = ctypes.c_int64
        L._shape_ready = True
    return L


def structure(circuit, n, arg=0, seed=0x5EED, **params):
    """The restated circuit's constraint structure (oracle/r1cs_shape.inc.c): a dict with per-constraint class
    `cls` (QUAD / LIN / COPY / CONST), support offsets `off` and signals `sup`, plus `_handle` for shape_map."""
    import numpy as np
    L = _shape_lib()
    _load_poseidon()
    p = CkParams(**params) if params else None
    st = CkStruct()
    rc = L.ck_structure(CIRCUITS[circuit], int(arg), ctypes.byref(p) if p is not None else None, int(n), seed,
                        ctypes.byref(st))
    if rc:
        raise RuntimeError("ck_structure(%s): %d" % (circuit, rc))
    nc, ns = st.n_cons, st.n_sup
    out = {"n_cons": nc,
           "cls": np.ctypeslib.as_array(st.cls, (nc,)).copy(),
           "off": np.ctypeslib.as_array(st.off, (nc + 1,)).copy(),
           "sup": np.ctypeslib.as_array(st.sup, (max(ns, 1),))[:ns].copy(),
           "_handle": st}
    return out


def shape_map(struct, n, n_protect, level):
    """-> (wit, witness_size): wit[s] = witness index of O0 signal s, -1 = removed (level 1: --O1-shaped, 2:
    --O2-shaped)."""
    import numpy as np
    wit = np.zeros(n, dtype=np.int32)
    m = _shape_lib().ck_shape_map(ctypes.byref(struct["_handle"]), n, n_protect, level, wit.ctypes.data)
    if m < 0:
        raise RuntimeError("ck_shape_map: %d" % m)
    return wit, int(m)


def free_structure(struct):
    _shape_lib().ck_struct_free(ctypes.byref(struct["_handle"]))
