"""Synthetic ICAO 9303 passports with a real EF.SOD: DER CMS SignedData over an LDSSecurityObject,
signed attributes, a document-signer certificate and the signature, plus DG1 and DG15.

The input side of the reference starts from such files ({dg1, dg15, sod} JSON, base64 fields;
test/process_passport.js:674-816 processPassport). This module makes them from seeded streams so
the SOD preprocessor (pzk_passport_parse / pzk_passport_inputs, include/pzkpassport.h) can be run
and checked in bulk; tools/gen_sod_fixtures.js runs the reference's own processPassport over the
same files to pin it. Layout of the DER (ICAO 9303-10 §4.6.2, RFC 5652):

  77 EF.SOD { ContentInfo SEQ { OID signedData, [0] { SignedData SEQ {
      INTEGER 3, SET { digest AlgId }, SEQ { OID ldsSecurityObject, [0] { OCTET STRING <EC> } },
      [0] { Certificate }, SET { SignerInfo SEQ { INTEGER 1, SEQ { issuer, serial },
      digest AlgId, [0] <signed attributes>, signature AlgId, OCTET STRING <signature> } } } } } }

  EC = LDSSecurityObject SEQ { INTEGER 0, hash AlgId, SEQ { SEQ { INTEGER dg, OCTET STRING H(dg) }... } }
  SA = SET { contentType, [signingTime], messageDigest = H(EC) }  (signed as the SET, stored as [0])
"""
import hashlib

from .field import SplitMix64
from .inputs import (BP256, BP384, P224, P256, Curve, EcKey, RsaKey, _dg15_rsa1024, _mrz_dg1, pkcs1v15_sha1_sign,
                     pkcs1v15_sha256_sign, pss_sign)

# secp521r1 (SEC 2 2.6.1): a named-curve key the reference recognises by name (getSigType :230, 66-bit chunks)
P521 = Curve("secp521r1", p=2 ** 521 - 1, a=2 ** 521 - 4,
             b=int("0051953EB9618E1C9A1F929A21A0B68540EEA2DA725B99B315F3B8B489918EF109E156193951EC7E937B1652C0BD3BB1BF07"
                   "3573DF883D2C34F1EF451FD46B503F00", 16),
             n=int("01FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFA51868783BF2F966B7FCC0148F709A5D03BB5C9B8"
                   "899C47AEBB6FB71E91386409", 16),
             g=(int("00C6858E06B70404E9CD9E3ECB662395B4429C648139053FB521F828AF606B4D3DBAA14B5E77EFE75928FE1DC127A2FFA8DE3348"
                    "B3C1856A429BF97E7E31C2E5BD66", 16),
                int("011839296A789A3BC0045C8A5FB42C7D1BD998F54449579B446817AFBD17273E662C97EE72995EF42640C550B9013FAD0761353C"
                    "7086A272C24088BE94769FD16650", 16)))
CURVE_OID = {"prime256v1": "1.2.840.10045.3.1.7", "secp521r1": "1.3.132.0.35"}

OID = {
    "sha1": "1.3.14.3.2.26", "sha224": "2.16.840.1.101.3.4.2.4", "sha256": "2.16.840.1.101.3.4.2.1",
    "sha384": "2.16.840.1.101.3.4.2.2", "sha512": "2.16.840.1.101.3.4.2.3",
    "rsaEncryption": "1.2.840.113549.1.1.1", "sha1WithRSAEncryption": "1.2.840.113549.1.1.5",
    "sha256WithRSAEncryption": "1.2.840.113549.1.1.11", "rsassaPss": "1.2.840.113549.1.1.10",
    "mgf1": "1.2.840.113549.1.1.8", "ecPublicKey": "1.2.840.10045.2.1", "primeField": "1.2.840.10045.1.1",
    "ecdsaWithSHA224": "1.2.840.10045.4.3.1", "ecdsaWithSHA256": "1.2.840.10045.4.3.2",
    "ecdsaWithSHA384": "1.2.840.10045.4.3.3", "signedData": "1.2.840.113549.1.7.2",
    "ldsSecurityObject": "2.23.136.1.1.1", "contentType": "1.2.840.113549.1.9.3",
    "messageDigest": "1.2.840.113549.1.9.4", "signingTime": "1.2.840.113549.1.9.5",
    "countryName": "2.5.4.6", "commonName": "2.5.4.3",
}
HASH_NAME = {160: "sha1", 224: "sha224", 256: "sha256", 384: "sha384", 512: "sha512"}


# ------------------------------------------------------------------------------ DER
def der_len(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def tlv(tag, body):
    return bytes([tag]) + der_len(len(body)) + body


def seq(*parts):
    return tlv(0x30, b"".join(parts))


def set_(*parts):
    return tlv(0x31, b"".join(parts))


def ctx(n, *parts):
    return tlv(0xA0 + n, b"".join(parts))


def integer(x):
    b = x.to_bytes(max(1, (x.bit_length() + 8) // 8), "big")  # one spare bit: non-negative two's complement
    return tlv(0x02, b)


def octets(b):
    return tlv(0x04, b)


def bitstring(b):
    return tlv(0x03, b"\x00" + b)


def null():
    return b"\x05\x00"


def oid(dotted):
    a = [int(x) for x in dotted.split(".")]
    out = bytearray([40 * a[0] + a[1]])
    for v in a[2:]:
        enc = [v & 0x7F]
        v >>= 7
        while v:
            enc.append(0x80 | (v & 0x7F))
            v >>= 7
        out += bytes(reversed(enc))
    return tlv(0x06, bytes(out))


def alg(name, params=None):
    return seq(oid(OID.get(name, name)), params if params is not None else null())


def name_(cn):
    return seq(set_(seq(oid(OID["countryName"]), tlv(0x13, b"UT"))), set_(seq(oid(OID["commonName"]), tlv(0x13, cn))))


def _fixed(x, n):
    return x.to_bytes(n, "big")


# ------------------------------------------------------------------------------ SOD parts
def lds_security_object(hash_bits, dgs):
    """LDSSecurityObject over [(dg_number, dg_bytes)] in the given order."""
    h = HASH_NAME[hash_bits]
    rows = [seq(integer(n), octets(hashlib.new(h, d).digest())) for n, d in dgs]
    return seq(integer(0), alg(h), seq(*rows))


def signed_attributes(ec, hash_bits, signing_time=b"240101120000Z"):
    """The SET the signer signs; messageDigest last (where processPassport's getZero looks, :322-358)."""
    attrs = [seq(oid(OID["contentType"]), set_(oid(OID["ldsSecurityObject"])))]
    if signing_time:
        attrs.append(seq(oid(OID["signingTime"]), set_(tlv(0x17, signing_time))))
    attrs.append(seq(oid(OID["messageDigest"]), set_(octets(hashlib.new(HASH_NAME[hash_bits], ec).digest()))))
    return set_(*attrs)


def rsa_spki(n, e):
    return seq(alg("rsaEncryption"), bitstring(seq(integer(n), integer(e))))


def ec_spki(curve, q):
    """Explicit-parameter EC key (processPassport reads curve.a: extract_ecdsa_pubkey :439-453)."""
    L = (curve.p.bit_length() + 7) // 8
    point = lambda pt: b"\x04" + _fixed(pt[0], L) + _fixed(pt[1], L)
    params = seq(integer(1), seq(oid(OID["primeField"]), integer(curve.p)),
                 seq(octets(_fixed(curve.a, L)), octets(_fixed(curve.b, L))), octets(point(curve.g)), integer(curve.n),
                 integer(1))
    return seq(seq(oid(OID["ecPublicKey"]), params), bitstring(point(q)))


def ec_spki_named(curve_name, curve, q):
    """Named-curve EC key: the parameters are an OID (extract_ecdsa_pubkey then takes the OID's name, :449-451)."""
    L = (curve.p.bit_length() + 7) // 8
    return seq(seq(oid(OID["ecPublicKey"]), oid(CURVE_OID[curve_name])),
               bitstring(b"\x04" + _fixed(q[0], L) + _fixed(q[1], L)))


def certificate(spki, sig_alg, rng):
    tbs = seq(ctx(0, integer(2)), integer(1 + rng.below(1 << 62)), sig_alg, name_(b"CSCA"),
              seq(tlv(0x17, b"230101000000Z"), tlv(0x17, b"330101000000Z")), name_(b"DS"), spki)
    return seq(tbs, sig_alg, bitstring(rng.bytes(256)))


def pss_alg(hash_bits, salt):
    h = alg(HASH_NAME[hash_bits])
    return alg("rsassaPss", seq(ctx(0, h), ctx(1, alg("mgf1", h)), ctx(2, integer(salt))))


def ef_sod(ec, sa, signature_field, spki, sig_alg, hash_bits, rng):
    """EF.SOD bytes: sa is the signed SET (tag 0x31), stored under [0] IMPLICIT in the SignerInfo."""
    dig = alg(HASH_NAME[hash_bits])
    signer = seq(integer(1), seq(name_(b"CSCA"), integer(7)), dig, b"\xa0" + sa[1:], sig_alg, octets(signature_field))
    sd = seq(integer(3), set_(dig), seq(oid(OID["ldsSecurityObject"]), ctx(0, octets(ec))),
             ctx(0, certificate(spki, sig_alg, rng)), set_(signer))
    return tlv(0x77, seq(oid(OID["signedData"]), ctx(0, sd)))


# ------------------------------------------------------------------------------ passports
SIG_KIND = {  # SIGNATURE_TYPE -> (key, sa / ec hash bits, scheme, salt)
    1: ("rsa2048", 256, "pkcs1", 0), 2: ("rsa4096", 256, "pkcs1", 0), 3: ("rsa2048", 160, "pkcs1", 0),
    10: ("rsa2048e3", 256, "pss", 32), 11: ("rsa2048", 256, "pss", 32), 12: ("rsa2048", 256, "pss", 64),
    13: ("rsa2048", 384, "pss", 48), 14: ("rsa3072", 256, "pss", 32), 20: ("p256", 256, "ecdsa", 0),
    21: ("bp256", 256, "ecdsa", 0), 24: ("p224", 224, "ecdsa", 0), 25: ("bp384", 384, "ecdsa", 0),
    27: ("p521", 256, "ecdsa", 0),
}


def signer_key(sig, seed=5, k=0):
    kind = SIG_KIND[sig][0]
    rng = SplitMix64((seed << 32) ^ (0x534F4400 + 16 * k + sig))
    if kind == "p256":
        return EcKey(rng, P256)
    if kind == "bp256":
        return EcKey(rng, BP256)
    if kind == "p521":
        return EcKey(rng, P521)
    if kind == "p224":
        return EcKey(rng, P224, hashlib.sha224)
    if kind == "bp384":
        return EcKey(rng, BP384, hashlib.sha384)
    bits = {"rsa2048": 2048, "rsa2048e3": 2048, "rsa4096": 4096, "rsa3072": 3072}[kind]
    return RsaKey(bits, rng, 3 if kind == "rsa2048e3" else 65537)


def make_passport(sig, key, index, seed=5, dg_hash=None, n_dgs=5, dg15=True, td1=False, signing_time=True,
                  named_curve=None, pss_salt_param=True, odd_dg1=False):
    """One synthetic passport: {dg1, dg15, sod} bytes plus the values the SOD carries (for checks).
    DG1 is hashed first in the LDS object and DG15 (when present) last, DGs 2, 11, 12, 14 between.
    Edge layouts: named_curve (an EC key named by OID), pss_salt_param=False (RSASSA-PSS parameters
    without saltLength), odd_dg1 (a DG11 hash first, then a DG2 entry whose 33-byte value holds DG1's
    digest one hex digit in: the reference's string search finds it there, a half-byte shift)."""
    _, hbits, scheme, salt = SIG_KIND[sig]
    dg_hash = dg_hash or hbits
    rng = SplitMix64((seed << 40) ^ (0x534F4450 + index))
    dg1 = _mrz_dg1(rng)
    if td1:
        dg1 = bytes.fromhex("615d5f1f5a") + dg1[5:95] + b"<<"  # TD1 DG1: 95 bytes
    d15 = _dg15_rsa1024(rng) if dg15 else b""
    others = [(n, rng.bytes(64 + rng.below(64))) for n in (2, 11, 12, 14)][:max(0, n_dgs - 1 - (1 if dg15 else 0))]
    dgs = [(1, dg1)] + others + ([(15, d15)] if dg15 else [])
    ec = lds_security_object(dg_hash, dgs)
    if odd_dg1:
        h = HASH_NAME[dg_hash]
        crafted = bytes.fromhex("0" + hashlib.new(h, dg1).hexdigest() + "0")
        rows = [seq(integer(11), octets(hashlib.new(h, others[0][1] if others else b"").digest())),
                seq(integer(2), octets(crafted))] + [seq(integer(n), octets(hashlib.new(h, d).digest())) for n, d in dgs]
        ec = seq(integer(0), alg(h), seq(*rows))
    sa = signed_attributes(ec, hbits, b"240101120000Z" if signing_time else None)
    hf = getattr(hashlib, HASH_NAME[hbits])
    if scheme == "ecdsa":
        r, s = key.sign(sa, rng)
        spki = ec_spki_named(named_curve, key.curve, key.q) if named_curve else ec_spki(key.curve, key.q)
        sig_field, sig_alg = seq(integer(r), integer(s)), alg("ecdsaWithSHA%d" % hbits, b"")
        signature = (r, s)
    else:
        if scheme == "pss":
            signature = pss_sign(key, sa, rng.bytes(salt), hf)
            sig_alg = pss_alg(hbits, salt) if pss_salt_param else alg("rsassaPss", seq(
                ctx(0, alg(HASH_NAME[hbits])), ctx(1, alg("mgf1", alg(HASH_NAME[hbits])))))
        else:
            signature = (pkcs1v15_sha1_sign if hbits == 160 else pkcs1v15_sha256_sign)(key, sa)
            sig_alg = alg("sha1WithRSAEncryption" if hbits == 160 else "sha256WithRSAEncryption")
        sig_field, spki = _fixed(signature, key.bits // 8), rsa_spki(key.n, key.e)
    sod = ef_sod(ec, sa, sig_field, spki, sig_alg, hbits, rng)
    return dict(dg1=dg1, dg15=d15, sod=sod, ec=ec, sa=sa, sig=signature, n=key.n, sig_type=sig)
