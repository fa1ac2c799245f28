"""ctypes binding of libpzkwit.so (include/pzkwit.h).

The library is the only compute path: there is no CPU fallback. Loading fails loudly
when the shared object is missing, and instance creation fails when no HIP device is
visible (PZK_E_NODEVICE).
"""
import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PZK_LIB selects another build of the same library (A/B builds under tools/gpu); default: the in-tree one
LIB_PATH = os.environ.get("PZK_LIB") or os.path.join(PKG, "lib", "libpzkwit.so")

PZK_CIRCUIT_REGISTER, PZK_CIRCUIT_POSEIDON, PZK_CIRCUIT_SHA256, PZK_CIRCUIT_SHA1 = 0, 1, 2, 3
PZK_CIRCUIT_SHA384, PZK_CIRCUIT_SHA512, PZK_CIRCUIT_QUERY = 4, 5, 6
PZK_EXEC_SYNC = 1

# C-ABI entry points declared in include/pzkwit.h and include/pzkpassport.h (checked by tests/test_capi.py)
EXPORTS = ("pzk_instance_create", "pzk_instance_destroy", "pzk_instance_info", "pzk_instance_input",
           "pzk_wtns_header", "pzk_witness_batch", "pzk_witness_batch_host", "pzk_instance_sync",
           "pzk_instance_create_mapped", "pzk_sym_check", "pzk_timing", "pzk_phase_info", "pzk_last_error",
           "pzk_version", "pzk_passport_parse", "pzk_passport_inputs")

STATUS_NAMES = {
    0: "OK", 1: "Num2Bits (bitify.circom:26)", 2: "AliasCheck (aliascheck.circom:14)",
    3: "IsZero (comparators.circom:20)", 4: "GetLastBitUnsecure (arithmetic.circom:169)",
    5: "GetLastNBits (arithmetic.circom:203)", 6: "Bits2 (sha2Common.circom:65)",
    7: "PassportVerificationBuilder (passportVerificationBuilder.circom:155)",
    8: "RsaVerifyPkcs1v15 (rsa.circom:48)", 9: "RsaVerifyPkcs1v15 (rsa.circom:53)",
    10: "RsaVerifyPkcs1v15 (rsa.circom:57)", 11: "BigMultModP (bigInt.circom:245)",
    12: "BigIntIsZero (bigIntComparators.circom:128)", 13: "SMTLevIns (SMTVerifier.circom:54)",
    14: "BabyjubjubAdd (babyjubjub/curve.circom:98)", 15: "BigModInv (bigInt.circom:364)",
    16: "verifyECDSABits (ecdsa.circom:81)", 17: "VerifyRsaPssSig (rsaPss.circom:73)",
    18: "VerifyRsaPssSig (rsaPss.circom:182)", 64: "input out of range",
}


class PzkParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "circuit", "size_arg", "signature_type", "dg_hash_type", "document_type", "ec_block_number",
        "ec_shift", "dg1_shift", "aa_signature_algo", "dg15_shift", "dg15_block_number", "aa_shift")]


class PzkInfo(ctypes.Structure):
    _fields_ = [("witness_size", ctypes.c_uint64), ("n_inputs", ctypes.c_uint64), ("n_outputs", ctypes.c_uint32),
                ("n_public_inputs", ctypes.c_uint32), ("n_input_groups", ctypes.c_uint32),
                ("pipeline_depth", ctypes.c_uint32)]


class PzkExec(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_int32), ("stream", ctypes.c_void_p)]


SINK_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                           ctypes.c_size_t, ctypes.c_void_p)


class PzkError(RuntimeError):
    pass


_PARAM_MAP = dict(sig="signature_type", dg_hash="dg_hash_type", doc="document_type", ec_blocks="ec_block_number",
                  ec_shift="ec_shift", dg1_shift="dg1_shift", aa="aa_signature_algo", dg15_shift="dg15_shift",
                  dg15_blocks="dg15_block_number", aa_shift="aa_shift")


def param_fields(params):
    """short names (inputs.CANONICAL) -> pzk_params field names"""
    return {_PARAM_MAP.get(k, k): int(v) for k, v in params.items()}


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PzkError("libpzkwit.so not built (%s): run __graft_entry__.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        L.pzk_instance_create.argtypes = [ctypes.POINTER(PzkParams), ctypes.POINTER(ctypes.c_void_p)]
        L.pzk_instance_destroy.argtypes = [ctypes.c_void_p]
        L.pzk_instance_destroy.restype = None
        L.pzk_instance_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(PzkInfo)]
        L.pzk_instance_input.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_char_p),
                                         ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.pzk_wtns_header.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.pzk_witness_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(PzkExec)]
        L.pzk_witness_batch_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.POINTER(PzkExec)]
        L.pzk_instance_sync.argtypes = [ctypes.c_void_p]
        L.pzk_witness_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, SINK_FN,
                                         ctypes.c_void_p, ctypes.POINTER(PzkExec)]
        L.pzk_instance_create_mapped.argtypes = [ctypes.POINTER(PzkParams), ctypes.c_char_p, ctypes.c_size_t,
                                                 ctypes.POINTER(ctypes.c_void_p)]
        L.pzk_sym_check.argtypes = [ctypes.POINTER(PzkParams), ctypes.c_char_p, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_uint64)]
        L.pzk_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
        L.pzk_phase_info.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint64)]
        L.pzk_layout_query.argtypes = [ctypes.POINTER(PzkParams), ctypes.POINTER(PzkInfo),
                                       ctypes.POINTER(ctypes.c_uint32)]
        L.pzk_layout_region.argtypes = [ctypes.POINTER(PzkParams), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        L.pzk_last_error.restype = ctypes.c_char_p
        L.pzk_version.restype = ctypes.c_char_p
        _lib = L
    return _lib


def layout_info(params, circuit=None, size_arg=0):
    """pzk_info of an instance (default: RegisterIdentityBuilder), from the host layout (no device)."""
    p = PzkParams(circuit=PZK_CIRCUIT_REGISTER if circuit is None else circuit, size_arg=size_arg)
    for k, v in param_fields(params).items():
        setattr(p, k, v)
    info = PzkInfo()
    _check(lib().pzk_layout_query(ctypes.byref(p), ctypes.byref(info), None))
    return info


def layout_witness_size(params, circuit=None):
    """Witness elements of a RegisterIdentityBuilder instance, from the host layout (no device)."""
    return int(layout_info(params, circuit).witness_size)


def layout_inputs(params, circuit=None):
    """Input elements (flat row length / 32) of a RegisterIdentityBuilder instance (no device)."""
    return int(layout_info(params, circuit).n_inputs)


def sym_check(params, sym, circuit=None, size_arg=0):
    """Validate a .sym text against an instance's O0 numbering (host only) -> mapped witness size."""
    p = PzkParams(circuit=PZK_CIRCUIT_REGISTER if circuit is None else circuit, size_arg=size_arg)
    for k, v in param_fields(params).items():
        setattr(p, k, v)
    b = sym.encode() if isinstance(sym, str) else sym
    n = ctypes.c_uint64()
    _check(lib().pzk_sym_check(ctypes.byref(p), b, len(b), ctypes.byref(n)))
    return int(n.value)


def _check(rc):
    if rc != 0:
        raise PzkError("pzkwit error %d: %s" % (rc, lib().pzk_last_error().decode()))


class Instance:
    """One compiled circuit instance (the analogue of circom's compiled WASM module)."""

    def __init__(self, circuit=PZK_CIRCUIT_REGISTER, size_arg=0, params=None, sym=None):
        """sym: optional signal -> witness map in circom .sym text (pzk_instance_create_mapped)."""
        L = lib()
        p = PzkParams(circuit=circuit, size_arg=size_arg)
        if params:
            m = dict(sig="signature_type", dg_hash="dg_hash_type", doc="document_type",
                     ec_blocks="ec_block_number", ec_shift="ec_shift", dg1_shift="dg1_shift",
                     aa="aa_signature_algo", dg15_shift="dg15_shift", dg15_blocks="dg15_block_number",
                     aa_shift="aa_shift")
            for k, v in params.items():
                setattr(p, m.get(k, k), int(v))
        h = ctypes.c_void_p()
        if sym is None:
            _check(L.pzk_instance_create(ctypes.byref(p), ctypes.byref(h)))
        else:
            b = sym.encode() if isinstance(sym, str) else sym
            _check(L.pzk_instance_create_mapped(ctypes.byref(p), b, len(b), ctypes.byref(h)))
        self._h = h
        info = PzkInfo()
        _check(L.pzk_instance_info(h, ctypes.byref(info)))
        self.witness_size = int(info.witness_size)
        self.n_inputs = int(info.n_inputs)
        self.n_outputs = int(info.n_outputs)
        self.n_public_inputs = int(info.n_public_inputs)
        self.input_groups = []
        for i in range(info.n_input_groups):
            nm, off, ln = ctypes.c_char_p(), ctypes.c_uint64(), ctypes.c_uint64()
            _check(L.pzk_instance_input(h, i, ctypes.byref(nm), ctypes.byref(off), ctypes.byref(ln)))
            self.input_groups.append((nm.value.decode(), int(off.value), int(ln.value)))

    def close(self):
        if getattr(self, "_h", None):
            lib().pzk_instance_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def wtns_header(self):
        h = (ctypes.c_uint8 * 76)()
        _check(lib().pzk_wtns_header(self._h, h))
        return bytes(h)

    def witness_batch_device(self, d_inputs, batch, d_wtns, stride, d_status=None, stream=None, device=-1, sync=False,
                             timing=False):
        """stream=None: pipelined on the instance's streams (complete after sync()); a stream
        handle: ordered after and joined into it. device -1 = the instance's device."""
        ex = PzkExec(device=device, flags=(PZK_EXEC_SYNC if sync else 0) | (2 if timing else 0), stream=stream)
        _check(lib().pzk_witness_batch(self._h, ctypes.c_void_p(d_inputs), batch, ctypes.c_void_p(d_wtns), stride,
                                       ctypes.c_void_p(d_status) if d_status else None, ctypes.byref(ex)))

    def sync(self):
        """Wait for every call issued on this instance (pzk_instance_sync)."""
        _check(lib().pzk_instance_sync(self._h))

    def timing(self, reset=False):
        """{phase: (ms accumulated, launches)} from calls made with timing=True (HIP events)."""
        cap = 32
        names = (ctypes.c_char_p * cap)()
        ms = (ctypes.c_double * cap)()
        n = (ctypes.c_uint64 * cap)()
        cnt = ctypes.c_uint32(cap)
        _check(lib().pzk_timing(self._h, names, ms, n, ctypes.byref(cnt), 1 if reset else 0))
        return {names[i].decode(): (ms[i], int(n[i])) for i in range(cnt.value)}

    def phase_info(self):
        """[(phase, kernel symbol, algorithmic bytes per witness)]"""
        out = []
        for p in range(32):
            nm, kn, b = ctypes.c_char_p(), ctypes.c_char_p(), ctypes.c_uint64()
            if lib().pzk_phase_info(self._h, p, ctypes.byref(nm), ctypes.byref(kn), ctypes.byref(b)) != 0:
                break
            out.append((nm.value.decode(), kn.value.decode(), int(b.value)))
        return out

    def witness_stream(self, inputs, sink, chunk=0):
        """Streamed delivery (pzk_witness_stream): sink(first, rows, status) gets numpy views of each chunk's
        pinned host rows ((n, W, 32) uint8) and statuses, valid only during the call; a truthy return stops."""
        a = np.ascontiguousarray(inputs, dtype=np.uint8)
        assert a.ndim == 3 and a.shape[1:] == (self.n_inputs, 32), a.shape
        W = self.witness_size
        err = []

        def _cb(user, first, n, rows, stride, status):
            try:
                r = np.ctypeslib.as_array(ctypes.cast(rows, ctypes.POINTER(ctypes.c_uint8)), shape=(n * stride,))
                s = np.ctypeslib.as_array(ctypes.cast(status, ctypes.POINTER(ctypes.c_int32)), shape=(n,))
                return 1 if sink(first, r.reshape(n, stride)[:, : 32 * W].reshape(n, W, 32), s) else 0
            except Exception as e:  # noqa: BLE001  (reported after the call)
                err.append(e)
                return 1
        cb = SINK_FN(_cb)
        ex = PzkExec(device=-1, flags=0, stream=None)
        rc = lib().pzk_witness_stream(self._h, a.ctypes.data, a.shape[0], chunk, cb, None, ctypes.byref(ex))
        if err:
            raise err[0]
        _check(rc)

    def witness_batch_host(self, inputs):
        """inputs: (batch, n_inputs, 32) uint8 -> (witness (batch, W, 32) uint8, status (batch,) int32)."""
        a = np.ascontiguousarray(inputs, dtype=np.uint8)
        if a.ndim == 2:
            a = a[None]
        b = a.shape[0]
        assert a.shape[1:] == (self.n_inputs, 32), a.shape
        out = np.empty((b, self.witness_size, 32), dtype=np.uint8)
        st = np.zeros(b, dtype=np.int32)
        ex = PzkExec(device=-1, flags=0, stream=None)
        _check(lib().pzk_witness_batch_host(self._h, a.ctypes.data, b, out.ctypes.data, st.ctypes.data,
                                            ctypes.byref(ex)))
        return out, st
