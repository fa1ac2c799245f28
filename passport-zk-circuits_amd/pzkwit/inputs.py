"""Caller-side data formats: SHA padding, bit arrays, limb chunking, synthetic
passports and packing of circuit inputs into the flat Fr buffer the C-ABI takes.

Mirrors the input preparation of test/process_passport.js (padding :11-91,
bigintToArrayString :125-135, getFakeIdenData :628-657, writeToJson :659-672).
Synthetic workloads follow SURVEY.md §8d (configs 2-4, seeds 0x2-0x4).
"""
import hashlib
import math
import os

import numpy as np

from .field import P, SplitMix64, poseidon

def process_pool(workers, initializer=None, initargs=()):
    """Worker pool for input generation. Spawned, not forked: a fork of a process that has
    initialised HIP (torch, libpzkwit) hands the children a runtime they cannot use, and the
    parent's device state must not be touched by them either."""
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor
    return ProcessPoolExecutor(workers, mp_context=multiprocessing.get_context("spawn"), initializer=initializer,
                               initargs=initargs)


# ----------------------------------------------------------- process_passport.js
def sha_pad(msg: bytes, block_bits=512) -> bytes:
    """padding() test/process_passport.js:11-91 (0x80, zeros, big-endian bit length)."""
    bs = block_bits // 8
    lsz = 8 if block_bits == 512 else 16
    padlen = (bs - ((len(msg) + 1 + lsz) % bs)) % bs
    return msg + b"\x80" + b"\x00" * padlen + (8 * len(msg)).to_bytes(lsz, "big")


def bits_msb_first(data: bytes):
    """bytes -> list of 0/1, MSB first per byte (process_passport.js:702-713)."""
    return np.unpackbits(np.frombuffer(data, dtype=np.uint8)).astype(np.uint8)


def padded_bits(msg: bytes, block_bits=512):
    """The bit array processPassport builds from padding()'s hex (process_passport.js:701-757):
    BigInt("0x" + padded).toString(2).split(""), then zeros prepended up to a multiple of the block
    length. Equal to the MSB-first bits of the padded message except when the padded message starts
    with a whole block of zero bits: the BigInt round trip drops it (reproduced, not fixed)."""
    bits = bits_msb_first(sha_pad(msg, block_bits))
    nz = np.flatnonzero(bits)
    sig = bits[nz[0]:] if nz.size else bits[:0]
    total = -(-len(sig) // block_bits) * block_bits if len(sig) % block_bits else len(sig)
    out = np.zeros(total, dtype=np.uint8)
    out[total - len(sig):] = sig
    return out


def fake_iden_data(ec: bytes, pk_hash: int):
    """getFakeIdenData (process_passport.js:628-657): skIdentity = the first 62 hex digits of
    SHA-256(EC) (as a hex string, leading zeros kept), the one-leaf SMT root Poseidon3(pkHash,
    pkHash, 1) as bare hex, 80 zero siblings. -> (sk_hex, root_hex, branches)."""
    sk_hex = hashlib.sha256(ec).hexdigest()[:62]
    return sk_hex, "%x" % poseidon([pk_hash, pk_hash, 1]), [0] * 80


def chunk_limbs(x: int, n=64, k=32):
    """bigintToArrayString(n, k, x) process_passport.js:125-135 (little-endian limbs)."""
    m = (1 << n) - 1
    return [(x >> (n * i)) & m for i in range(k)]


# ------------------------------------------------------------------ RSA (synthetic)
_SMALL_PRIMES = [p for p in range(3, 2000) if all(p % q for q in range(2, int(p ** 0.5) + 1))]


def _is_probable_prime(n, rng):
    for q in _SMALL_PRIMES:
        if n % q == 0:
            return n == q
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(16):
        a = 2 + rng.below(n - 3)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _gen_prime(bits, rng):
    while True:
        c = rng.bits(bits) | (3 << (bits - 2)) | 1
        if _is_probable_prime(c, rng):
            return c


class RsaKey:
    def __init__(self, bits, rng, e=65537):
        while True:
            p = _gen_prime(bits // 2, rng)
            q = _gen_prime(bits // 2, rng)
            if p == q:
                continue
            n = p * q
            phi = (p - 1) * (q - 1)
            if n.bit_length() != bits or math.gcd(phi, e) != 1:
                continue
            break
        self.n, self.e, self.p, self.q = n, e, p, q
        self.d = pow(e, -1, phi)
        self.dp, self.dq, self.qinv = self.d % (p - 1), self.d % (q - 1), pow(q, -1, p)
        self.bits = bits

    def sign_raw(self, m):
        s1 = pow(m, self.dp, self.p)
        s2 = pow(m, self.dq, self.q)
        h = (self.qinv * (s1 - s2)) % self.p
        return s2 + h * self.q


_DIGESTINFO_SHA256 = bytes.fromhex("3031300d060960864801650304020105000420")


_DIGESTINFO_SHA1 = bytes.fromhex("3021300906052b0e03021a05000414")


def pkcs1v15_sha1_sign(key: RsaKey, msg: bytes) -> int:
    """RSASSA-PKCS1-v1_5 with SHA-1 (SIGNATURE_TYPE 3, rsa.circom:73-109)."""
    return _pkcs1v15_sign(key, _DIGESTINFO_SHA1 + hashlib.sha1(msg).digest())


def pkcs1v15_sha256_sign(key: RsaKey, msg: bytes) -> int:
    return _pkcs1v15_sign(key, _DIGESTINFO_SHA256 + hashlib.sha256(msg).digest())


def _pkcs1v15_sign(key: RsaKey, t: bytes) -> int:
    k = key.bits // 8
    em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    return key.sign_raw(int.from_bytes(em, "big"))


def mgf1(seed: bytes, length: int, hf=hashlib.sha256) -> bytes:
    """MGF1 (RFC 8017 B.2.1) over hash hf."""
    out, n = b"", hf().digest_size
    for c in range((length + n - 1) // n):
        out += hf(seed + c.to_bytes(4, "big")).digest()
    return out[:length]


def mgf1_sha256(seed: bytes, length: int) -> bytes:
    return mgf1(seed, length, hashlib.sha256)


def pss_salt_len(sig):
    """SALT_LEN of VerifyRsaPssSig for SIGNATURE_TYPE 10-14 (signatureVerification.circom:46-75)."""
    return 64 if sig == 12 else 48 if sig == 13 else 32


def pss_sign(key: RsaKey, msg: bytes, salt: bytes, hf=hashlib.sha256) -> int:
    """RSASSA-PSS (RFC 8017 9.1.1) with hash hf and MGF1 over hf, emBits = modBits - 1."""
    h = hf(msg).digest()
    em_len = key.bits // 8
    hh = hf(b"\x00" * 8 + h + salt).digest()
    db = b"\x00" * (em_len - len(salt) - len(h) - 2) + b"\x01" + salt
    masked = bytes(a ^ b for a, b in zip(db, mgf1(hh, len(db), hf)))
    masked = bytes([masked[0] & 0x7F]) + masked[1:]
    return key.sign_raw(int.from_bytes(masked + hh + b"\xbc", "big"))


def pss_sha256_sign(key: RsaKey, msg: bytes, salt: bytes) -> int:
    return pss_sign(key, msg, salt, hashlib.sha256)


# -------------------------------------------------------------- ECDSA (synthetic)
class Curve:
    """Short-Weierstrass curve y^2 = x^3 + a x + b over F_p with generator g of order n."""

    def __init__(self, name, p, a, b, n, g):
        self.name, self.p, self.a, self.b, self.n, self.g = name, p, a, b, n, g

    def add(self, p1, p2):
        """Affine addition (None = point at infinity)."""
        if p1 is None:
            return p2
        if p2 is None:
            return p1
        P = self.p
        (x1, y1), (x2, y2) = p1, p2
        if x1 == x2:
            if (y1 + y2) % P == 0:
                return None
            lam = (3 * x1 * x1 + self.a) * pow(2 * y1, -1, P) % P
        else:
            lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
        x3 = (lam * lam - x1 - x2) % P
        return x3, (lam * (x1 - x3) - y1) % P

    def mul(self, k, pt=None):
        pt = self.g if pt is None else pt
        r = None
        for i in reversed(range(k.bit_length())):
            r = self.add(r, r)
            if (k >> i) & 1:
                r = self.add(r, pt)
        return r


# secp256r1, FIPS 186-4 D.1.2.3 (signatureVerification.circom:177-182 passes its A, B, P as 4 x 64-bit limbs)
P256 = Curve("secp256r1",
             p=0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF,
             a=0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFC,
             b=0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B,
             n=0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551,
             g=(0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
                0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5))
# brainpoolP256r1, RFC 5639 3.4 (signatureVerification.circom:191-196)
BP256 = Curve("brainpoolP256r1",
              p=0xA9FB57DBA1EEA9BC3E660A909D838D726E3BF623D52620282013481D1F6E5377,
              a=0x7D5A0975FC2C3057EEF67530417AFFE7FB8055C126DC5C6CE94A4B44F330B5D9,
              b=0x26DC5C6CE94A4B44F330B5D9BBD77CBF958416295CF7E1CE6BCCDC18FF8C07B6,
              n=0xA9FB57DBA1EEA9BC3E660A909D838D718C397AA3B561A6F7901E0E82974856A7,
              g=(0x8BD2AEB9CB7E57CB2C4B482FFC81B7AFB9DE27E1E3BD23C23A4453BD9ACE3262,
                 0x547EF835C3DAC4FD97F8461A14611DC9C27745132DED8E545C1D54C72F046997))
# secp224r1, FIPS 186-4 D.1.2.2 (SIGNATURE_TYPE 24: 7 x 32-bit chunks, signatureVerification.circom:230-243)
P224 = Curve("secp224r1",
             p=0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF000000000000000000000001,
             a=0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFE,
             b=0xB4050A850C04B3ABF54132565044B0B7D7BFD8BA270B39432355FFB4,
             n=0xFFFFFFFFFFFFFFFFFFFFFFFFFFFF16A2E0B8F03E13DD29455C5C2A3D,
             g=(0xB70E0CBD6BB4BF7F321390B94A03C1D356C21122343280D6115C1D21,
                0xBD376388B5F723FB4C22DFE6CD4375A05A07476444D5819985007E34))
# brainpoolP384r1, RFC 5639 3.6 (SIGNATURE_TYPE 25: 6 x 64-bit chunks, signatureVerification.circom:245-258)
BP384 = Curve("brainpoolP384r1",
              p=0x8CB91E82A3386D280F5D6F7E50E641DF152F7109ED5456B412B1DA197FB71123ACD3A729901D1A71874700133107EC53,
              a=0x7BC382C63D8C150C3C72080ACE05AFA0C2BEA28E4FB22787139165EFBA91F90F8AA5814A503AD4EB04A8C7DD22CE2826,
              b=0x04A8C7DD22CE28268B39B55416F0447C2FB77DE107DCD2A62E880EA53EEB62D57CB4390295DBC9943AB78696FA504C11,
              n=0x8CB91E82A3386D280F5D6F7E50E641DF152F7109ED5456B31F166E6CAC0425A7CF3AB6AF6B7FC3103B883202E9046565,
              g=(0x1D1C64F068CF45FFA2A63A81B7C13F6B8847A3E77EF14FE3DB7FCAFE0CBD10E8E826E03436D646AAEF87B2E247D4AF1E,
                 0x8ABE1D7520F9C2A45CB1EB8E95CFD55262B70B29FEEC5864E19C054FF99129280E4646217791811142820341263C5315))
EC_CURVES = {20: P256, 21: BP256, 24: P224, 25: BP384}  # SIGNATURE_TYPE -> curve
# SIGNATURE_TYPE -> (CHUNK_NUMBER, CHUNK_SIZE) of the ECDSA inputs and templates (registerIdentityBuilder.circom:81-99).
# 22 (brainpoolP320r1, 5 x 64) and 23 (secp192r1, 3 x 64) read hashed[] out of bounds in verifyECDSABits
# (ecdsa.circom:31-37: CHUNK_NUMBER x CHUNK_SIZE = 320 / 192 bits of a 256 / 160-bit hash): no circuit compiles.
EC_CHUNKS = {20: (4, 64), 21: (4, 64), 24: (7, 32), 25: (6, 64)}

P256_P, P256_A, P256_N, P256_G = P256.p, P256.a, P256.n, P256.g


def p256_add(p1, p2):
    return P256.add(p1, p2)


def p256_mul(k, pt=P256_G):
    return P256.mul(k, pt)


class EcKey:
    """ECDSA signer key (SIG 20: P-256, 21: brainpoolP256r1, 24: P-224 with SHA-224, 25: brainpoolP384r1 with SHA-384)."""

    def __init__(self, rng, curve=P256, hash_fn=None):
        self.curve = curve
        self.hash_fn = hash_fn or hashlib.sha256
        self.d = 1 + rng.below(curve.n - 1)
        self.q = curve.mul(self.d)
        self.n = self.q  # the "pubkey" of the passport dict: (x, y)

    def sign(self, msg: bytes, rng):
        """ECDSA (r, s) over the instance's hash; h = the digest as an integer, not reduced (ecdsa.circom:30-38:
        its CHUNK_NUMBER x CHUNK_SIZE bits are exactly the hash's)."""
        c = self.curve
        h = int.from_bytes(self.hash_fn(msg).digest(), "big")
        while True:
            k = 1 + rng.below(c.n - 1)
            r = c.mul(k)[0] % c.n
            s = pow(k, -1, c.n) * (h + r * self.d) % c.n
            if r and s:
                return r, s


def ecdsa_pk_hash(q, field_bits=256):
    """Poseidon2 of the low min(EC_FIELD_SIZE, 248) bits of x and y (passportVerificationBuilder.circom:193-230)."""
    m = (1 << min(field_bits, 248)) - 1
    return poseidon([q[0] & m, q[1] & m])


def sig_hash_type(sig):
    """HASH_TYPE of the signed attributes / encapsulated content (registerIdentityBuilder.circom:54-99)."""
    return 160 if sig in (3, 4) else 384 if sig in (13, 25) else 224 if sig == 24 else 256


def ec_hash_type(sig):
    """EC_HASH_TYPE, the encapsulated content's hash (passportVerificationBuilder.circom:53-59): HASH_TYPE as set
    before SIG 24 switches it to 224, so SHA-256 for SIG 24."""
    return 256 if sig == 24 else sig_hash_type(sig)


def hash_block(algo):
    """Block size in bits of the hash algo (DG_HASH_BLOCK_SIZE / HASH_BLOCK_SIZE, registerIdentityBuilder.circom:95-102)."""
    return 1024 if algo > 256 else 512


HASHES = {160: hashlib.sha1, 224: hashlib.sha224, 256: hashlib.sha256, 384: hashlib.sha384, 512: hashlib.sha512}


def sig_input_len(sig):
    """signature / pubkey input lengths (registerIdentityBuilder.circom:131-140)."""
    return 2 * EC_CHUNKS[sig][0] if sig >= 20 else 64 if sig == 2 else 48 if sig in (4, 14) else 32


def sig_limbs(v, sig):
    """RSA: integer -> K 64-bit limbs; ECDSA: (a, b) -> 2 x CHUNK_NUMBER chunks of CHUNK_SIZE bits
    (process_passport.js:125-135)."""
    if sig >= 20:
        k, n = EC_CHUNKS[sig]
        return chunk_limbs(v[0], n, k) + chunk_limbs(v[1], n, k)
    return chunk_limbs(v, 64, sig_input_len(sig))


# ------------------------------------------------------------- synthetic passports
CANONICAL = dict(sig=1, dg_hash=256, doc=3, ec_blocks=4, ec_shift=600, dg1_shift=248, aa=1,
                 dg15_shift=1496, dg15_blocks=3, aa_shift=256)  # hardhat.config.ts:30


def instance_params(sig):
    """The canonical instance with SIGNATURE_TYPE sig (SIG 3 / 4 hash with SHA-1 and need DG_HASH_TYPE 160).
    SIG 13 hashes with SHA-384 in 1024-bit blocks: DG_HASH_TYPE 384, and the block counts / EC_SHIFT the
    synthetic messages fit (EC and the RSA-1024 DG15 pad to 2 blocks; the SA, one block, holds at most 111 bytes)."""
    if sig in (13, 25):  # SHA-384 EC / SA hashers (SIG 25: ECDSA brainpoolP384r1)
        return dict(CANONICAL, sig=sig, dg_hash=384, ec_blocks=2, dg15_blocks=2, ec_shift=336)
    return dict(CANONICAL, sig=sig, dg_hash=160 if sig in (3, 4) else 224 if sig == 24 else 256)

_MRZ = b"ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789<"
_DG15_PREFIX = bytes.fromhex("6f81a230819f300d06092a864886f70d010101050003818d00308189028181")


def _mrz_dg1(rng):
    body = bytes(_MRZ[rng.below(len(_MRZ))] for _ in range(88))
    return bytes.fromhex("615b5f1f58") + body  # TD3 DG1: 93 bytes


def _dg15_rsa1024(rng):
    mod = bytearray(rng.bytes(128))
    mod[0] |= 0x80
    # 32-byte DER prefix puts the modulus at bit 256 = AA_SHIFT (identity.circom:34)
    return _DG15_PREFIX + b"\x00" + bytes(mod) + bytes.fromhex("0203010001")


def _keygen(args):
    seed, k, bits = args[:3]
    e = args[3] if len(args) > 3 else 65537
    rng = SplitMix64((seed << 32) ^ (0x4B455900 + k))
    if bits == "p256":
        return EcKey(rng)
    if bits == "bp256":
        return EcKey(rng, BP256)
    if bits == "p224":
        return EcKey(rng, P224, hashlib.sha224)
    if bits == "bp384":
        return EcKey(rng, BP384, hashlib.sha384)
    return RsaKey(bits, rng, e)


class PassportGen:
    """Synthetic passports for the canonical instance.

    Signer key k and passport i each draw from their own SplitMix64 stream, so any index
    range can be generated independently (sharded across ranks / worker processes)."""

    _shared = {}

    def __init__(self, seed=3, n_keys=64, key_bits=2048, params=None, workers=None, keys=None):
        self.seed = seed
        self.rng = SplitMix64(seed)
        self.params = dict(CANONICAL if params is None else params)
        self._pkhash = {}
        if keys is not None:  # signer keys made elsewhere (worker processes get the parent's)
            self.keys = list(keys)
            return
        if self.params["sig"] >= 20:
            key_bits = {20: "p256", 21: "bp256", 24: "p224", 25: "bp384"}[self.params["sig"]]
        elif self.params["sig"] == 2 and key_bits == 2048:
            key_bits = 4096
        elif self.params["sig"] in (4, 14) and key_bits == 2048:
            key_bits = 3072
        e = 3 if self.params["sig"] == 10 else 37187 if self.params["sig"] == 4 else 65537  # SIG 10: e = 3, SIG 4: 37187
        jobs = [(seed, k, key_bits) if e == 65537 else (seed, k, key_bits, e) for k in range(n_keys)]
        workers = workers or min(16, os.cpu_count() or 1)
        if n_keys >= 8 and workers > 1:
            with process_pool(min(workers, n_keys)) as ex:
                self.keys = list(ex.map(_keygen, jobs))
        else:
            self.keys = [_keygen(j) for j in jobs]

    @classmethod
    def shared(cls, seed=3, n_keys=64, sig=1):
        key = (seed, n_keys, sig)
        if key not in cls._shared:
            cls._shared[key] = cls(seed, n_keys, params=instance_params(sig))
        return cls._shared[key]

    @classmethod
    def install_shared(cls, seed, n_keys, sig, keys):
        """Pool initializer: the parent's signer keys, so workers do not regenerate them."""
        cls._shared[(seed, n_keys, sig)] = cls(seed, n_keys, params=instance_params(sig), keys=keys)

    @property
    def n_inputs(self):
        pr = self.params
        K = sig_input_len(pr["sig"])
        bs = hash_block(sig_hash_type(pr["sig"]))
        return 1 + pr["ec_blocks"] * bs + 1024 + pr["dg15_blocks"] * bs + 1024 + 2 * K + 80 + 1

    def passport_at(self, i, smt_depth=0, smt_root=False):
        """Passport i from its own stream (independent of generation order)."""
        saved = self.rng
        self.rng = SplitMix64((self.seed << 40) ^ (0x50415353 + i))
        try:
            return self.passport(i, smt_depth, smt_root)
        finally:
            self.rng = saved

    def pk_hash(self, key):
        """RSA pubkey hash = Poseidon5 of 5 x 192-bit limb triples (passportVerificationBuilder.circom:182-191);
        ECDSA: ecdsa_pk_hash."""
        h = self._pkhash.get(key.n)
        if h is None:
            if isinstance(key, EcKey):
                h = ecdsa_pk_hash(key.q, key.curve.p.bit_length())  # EC_FIELD_SIZE = CHUNK_NUMBER x CHUNK_SIZE
            else:
                a = chunk_limbs(key.n, 64, 15)
                h = poseidon([(a[3 * i] << 128) + (a[3 * i + 1] << 64) + a[3 * i + 2] for i in range(5)])
            self._pkhash[key.n] = h
        return h

    def passport(self, i, smt_depth=0, smt_root=False):
        """Returns dict of raw fields for passport i (bytes + ints). smt_depth k > 0: siblings[0..k-1] uniform
        non-zero Fr; the root is then computed (smt_root=True, Python Poseidon, ~0.6 ms
        per level) or left 0 (the circuit does not enforce it: passportVerificationBuilder.circom:240)."""
        pr = self.params
        rng = self.rng
        key = self.keys[i % len(self.keys)]
        dg1 = _mrz_dg1(rng)
        dg15 = _dg15_rsa1024(rng)
        # DG hashes: DG_HASH_TYPE; EC / SA hashes: HASH_TYPE (SHA-1 for SIG 3 / 4, SHA-384 for SIG 13,
        # passportVerificationBuilder.circom:16-59), whose block size sets the EC length (it pads to ec_blocks blocks)
        ht = sig_hash_type(pr["sig"])
        bs = hash_block(ht) // 8
        ec_len = 219 + rng.below(pr["ec_blocks"] * bs - (bs // 8 + 1) - 219 + 1)
        ec = bytearray(rng.bytes(ec_len))
        dgh, sah, ech = HASHES[pr["dg_hash"]], HASHES[ht], HASHES[ec_hash_type(pr["sig"])]
        h1, h15 = dgh(dg1).digest(), dgh(dg15).digest()
        d1 = pr["dg1_shift"] // 8
        ec[d1 - 7:d1] = bytes.fromhex("302502010104") + bytes([max(32, len(h1))])
        ec[d1:d1 + len(h1)] = h1
        d15 = pr["dg15_shift"] // 8
        ec[d15 - 7:d15] = bytes.fromhex("302502010f04") + bytes([max(32, len(h15))])
        ec[d15:d15 + len(h15)] = h15
        ec = bytes(ec)
        sa_shift = pr["ec_shift"] // 8
        hl = max(32, sah().digest_size)
        sa_max = 119 if bs == 64 else 111  # two 512-bit blocks, or one 1024-bit block (SHA-384)
        sa_len = sa_shift + hl + rng.below(sa_max - (sa_shift + hl) + 1)
        sa = bytearray(rng.bytes(sa_len))
        sa[sa_shift - 2:sa_shift] = bytes([0x04, hl])
        sa[sa_shift:sa_shift + hl] = (ech(ec).digest() + bytes(32))[:hl]
        sa = bytes(sa)
        if isinstance(key, EcKey):
            sig = key.sign(sa, rng)
        elif 10 <= pr["sig"] <= 14:
            sig = pss_sign(key, sa, rng.bytes(pss_salt_len(pr["sig"])), sah)
        elif pr["sig"] in (3, 4):
            sig = pkcs1v15_sha1_sign(key, sa)
        else:
            sig = pkcs1v15_sha256_sign(key, sa)
        pkh = self.pk_hash(key)
        sk_hex, root_hex, _ = fake_iden_data(ec, pkh)  # getFakeIdenData :628-657
        sk = int(sk_hex, 16)
        siblings = [0] * 80
        if smt_depth:
            for k in range(smt_depth):
                v = 0
                while v == 0:
                    v = rng.fr()
                siblings[k] = v
            root = None  # not enforced by the circuit
            if smt_root:
                from .query import smt_root as _root
                root = _root(pkh, pkh, siblings)  # SMTVerifier.circom:109-176 with key = value = pubkeyHash
        else:
            root = int(root_hex, 16)
        return dict(dg1=dg1, dg15=dg15, ec=ec, sa=sa, sig=sig, n=key.n, sk=sk, root=root,
                    siblings=siblings, pk_hash=pkh)


def passport_json(pp, params=CANONICAL):
    """The reference's input JSON (writeToJson, process_passport.js:659-672)."""
    sg = params["sig"]
    hb, db = hash_block(sig_hash_type(sg)), hash_block(params["dg_hash"])

    def bits(b, nbits, block):
        arr = padded_bits(b, block)
        assert len(arr) == nbits, (len(arr), nbits)
        return [str(int(x)) for x in arr]

    return {
        "dg1": bits(pp["dg1"], 1024, db),
        "dg15": bits(pp["dg15"], params["dg15_blocks"] * hb, db) if params["dg15_blocks"] else [],
        "signedAttributes": bits(pp["sa"], 1024, hb),
        "encapsulatedContent": bits(pp["ec"], params["ec_blocks"] * hb, hb),
        "pubkey": [str(x) for x in sig_limbs(pp["n"], sg)],
        "signature": [str(x) for x in sig_limbs(pp["sig"], sg)],
        "skIdentity": "0x%062x" % pp["sk"],  # getFakeIdenData's 62 hex digits, leading zeros kept
        "slaveMerkleRoot": hex(pp["root"] or 0),
        "slaveMerkleInclusionBranches": [str(x) for x in pp["siblings"]],
    }


def pack_register_inputs(pp, params=CANONICAL, out=None):
    """Flat input buffer in witness order: slaveMerkleRoot, encapsulatedContent, dg1, dg15,
    signedAttributes, signature, pubkey, slaveMerkleInclusionBranches, skIdentity
    (registerIdentityBuilder.circom:143-152, public input first). -> (nIn, 32) uint8."""
    K = sig_input_len(params["sig"])
    hb, db = hash_block(sig_hash_type(params["sig"])), hash_block(params["dg_hash"])
    ecL, d15L = params["ec_blocks"] * hb, params["dg15_blocks"] * hb
    n_in = 1 + ecL + 1024 + d15L + 1024 + 2 * K + 80 + 1
    buf = out if out is not None else np.zeros((n_in, 32), dtype=np.uint8)
    buf[:] = 0
    o = 0

    def put_int(v):
        nonlocal o
        buf[o] = np.frombuffer(int(v % P).to_bytes(32, "little"), dtype=np.uint8)
        o += 1

    def put_bits(b, nbits, block):
        nonlocal o
        if nbits == 0:
            return
        arr = padded_bits(b, block)
        if len(arr) != nbits:
            raise ValueError("padded length %d != %d bits" % (len(arr), nbits))
        buf[o:o + nbits, 0] = arr
        o += nbits

    def put_u64s(vals):
        nonlocal o
        for v in vals:
            buf[o, :8] = np.frombuffer(int(v).to_bytes(8, "little"), dtype=np.uint8)
            o += 1

    put_int(pp["root"] or 0)
    put_bits(pp["ec"], ecL, hb)  # the message each field's hasher reads, padded for that hash
    put_bits(pp["dg1"], 1024, db)
    put_bits(pp["dg15"], d15L, db)
    put_bits(pp["sa"], 1024, hb)
    put_u64s(sig_limbs(pp["sig"], params["sig"]))
    put_u64s(sig_limbs(pp["n"], params["sig"]))
    for s in pp["siblings"]:
        put_int(s)
    put_int(pp["sk"])
    assert o == n_in
    return buf


def sha256_config2_batch(batch, seed=2, blocks=6):
    """Config 2: messages of L in [312,375] bytes, padded to 6 blocks; -> (msgs, (batch, 3072, 32) uint8)."""
    rng = SplitMix64(seed)
    lo, hi = 64 * (blocks - 1) - 8, 64 * blocks - 9
    out = np.zeros((batch, 512 * blocks, 32), dtype=np.uint8)
    msgs = []
    for b in range(batch):
        L = lo + rng.below(hi - lo + 1)
        m = rng.bytes(L)
        msgs.append(m)
        out[b, :, 0] = bits_msb_first(sha_pad(m, 512))
    return msgs, out
