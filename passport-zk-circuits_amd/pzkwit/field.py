"""BN254 Fr helpers for the host side (input preparation), plus a host Poseidon.

The host Poseidon follows poseidon.circom:80-209 (same optimised constant set,
loaded from data/poseidon_t2_6.bin). It is used only by input preparation —
e.g. the fake identity root Poseidon3(pkHash, pkHash, 1) that
test/process_passport.js:628-657 (getFakeIdenData) computes on the host. The
witness itself is always computed on the GPU.
"""
import os
import struct

P = 21888242871839275222246405745257275088548364400416034343698204186575808495617
DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")
POSEIDON_BIN = os.path.join(DATA, "poseidon_t2_6.bin")

_params = None


def load_poseidon_params(path=POSEIDON_BIN):
    """-> {t: (nRP, C, M, P, S)}; M/P as row-major lists of lists."""
    global _params
    if _params is not None and path == POSEIDON_BIN:
        return _params
    with open(path, "rb") as f:
        raw = f.read()
    if raw[:8] != b"PZKPOS01":
        raise ValueError("bad Poseidon parameter file")
    off = 8
    (nt,) = struct.unpack_from("<I", raw, off)
    off += 4
    out = {}

    def elems(n):
        nonlocal off
        vals = [int.from_bytes(raw[off + 32 * i: off + 32 * i + 32], "little") for i in range(n)]
        off += 32 * n
        return vals

    for _ in range(nt):
        t, nrp, nc, ns = struct.unpack_from("<4I", raw, off)
        off += 16
        C = elems(nc)
        Mf = elems(t * t)
        Pf = elems(t * t)
        S = elems(ns)
        out[t] = (nrp, C, [Mf[i * t:(i + 1) * t] for i in range(t)], [Pf[i * t:(i + 1) * t] for i in range(t)], S)
    if path == POSEIDON_BIN:
        _params = out
    return out


def poseidon(inputs):
    """PoseidonHash(n) (poseidon.circom:214-226) on python ints."""
    t = len(inputs) + 1
    nrp, C, M, Pm, S = load_poseidon_params()[t]
    st = [0] + [x % P for x in inputs]
    st = [(st[i] + C[i]) % P for i in range(t)]

    def mix(state, mat):
        return [sum(mat[j][i] * state[j] for j in range(t)) % P for i in range(t)]

    for r in range(3):
        st = [pow(x, 5, P) for x in st]
        st = [(st[i] + C[(r + 1) * t + i]) % P for i in range(t)]
        st = mix(st, M)
    st = [pow(x, 5, P) for x in st]
    st = [(st[i] + C[4 * t + i]) % P for i in range(t)]
    st = mix(st, Pm)
    for r in range(nrp):
        s0 = (pow(st[0], 5, P) + C[5 * t + r]) % P
        base = (2 * t - 1) * r
        new0 = (S[base] * s0 + sum(S[base + i] * st[i] for i in range(1, t))) % P
        st = [new0] + [(st[i] + s0 * S[base + t + i - 1]) % P for i in range(1, t)]
    for r in range(3):
        st = [pow(x, 5, P) for x in st]
        st = [(st[i] + C[5 * t + nrp + r * t + i]) % P for i in range(t)]
        st = mix(st, M)
    st = [pow(x, 5, P) for x in st]
    return sum(M[j][0] * st[j] for j in range(t)) % P


class SplitMix64:
    """Deterministic generator used for every synthetic workload (SURVEY.md §8d seeds)."""

    M64 = (1 << 64) - 1

    def __init__(self, seed):
        self.s = seed & self.M64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & self.M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.M64
        return z ^ (z >> 31)

    def below(self, n):
        return self.next() % n

    def bytes(self, n):
        out = bytearray()
        while len(out) < n:
            out += self.next().to_bytes(8, "little")
        return bytes(out[:n])

    def fr(self):
        while True:
            x = self.next() | (self.next() << 64) | (self.next() << 128) | (self.next() << 192)
            if x < P:
                return x

    def bits(self, k):
        x = 0
        for i in range(0, k, 64):
            x |= self.next() << i
        return x & ((1 << k) - 1)
