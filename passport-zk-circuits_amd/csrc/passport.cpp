// Host-side bulk SOD preprocessor (include/pzkpassport.h).
//
// Restates test/process_passport.js:157-816 (processPassport and the extractors it calls) over a DER
// tree with the semantics of the reference's decoder, test/asn1.js (ASN1.decode :3520-3589 with its
// BIT / OCTET STRING encapsulation attempt, content() :3387-3450, toHexString :3499, simplifyASN1
// :3593-3606), so every walk the reference makes over `decoded(json.sod)` lands on the same element.
// Pinned by tests/golden/sod_vectors.json: the reference's processPassport itself, run on Node 12 over
// synthetic EF.SOD files (tools/gen_sod_fixtures.*).
#include <sched.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pzkpassport.h"

namespace pzk {
int api_fail(int code, const std::string& msg);  // runtime.cpp: sets pzk_last_error()
}

namespace {

struct Fail : std::runtime_error {
  int code;
  Fail(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
[[noreturn]] void fail(const std::string& m, int code = PZK_PP_PARSE) { throw Fail(code, m); }

// ------------------------------------------------------------------------------------ hashes
// computeHash (process_passport.js:93-111): SHA-1 / 224 / 256 / 384 / 512 selected by output length
inline uint32_t rol(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }
inline uint32_t ror(uint32_t x, int s) { return (x >> s) | (x << (32 - s)); }
inline uint64_t ror64(uint64_t x, int s) { return (x >> s) | (x << (64 - s)); }

std::vector<uint8_t> md_pad(const uint8_t* m, size_t n, size_t block, size_t lenbytes) {
  std::vector<uint8_t> p;
  p.reserve(n + block + lenbytes);
  p.assign(m, m + n);
  p.push_back(0x80);
  while ((p.size() + lenbytes) % block) p.push_back(0);
  for (size_t i = lenbytes; i-- > 0;) p.push_back(i >= 8 ? 0 : (uint8_t)((uint64_t)n * 8 >> (8 * i)));
  return p;
}

std::vector<uint8_t> sha1(const uint8_t* m, size_t n) {
  uint32_t h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
  const std::vector<uint8_t> p = md_pad(m, n, 64, 8);
  for (size_t o = 0; o < p.size(); o += 64) {
    uint32_t w[80];
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[o + 4 * i] << 24 | p[o + 4 * i + 1] << 16 | p[o + 4 * i + 2] << 8 | p[o + 4 * i + 3];
    for (int i = 16; i < 80; i++) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; i++) {
      uint32_t f, k;
      if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999; }
      else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1; }
      else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDC; }
      else { f = b ^ c ^ d; k = 0xCA62C1D6; }
      const uint32_t t = rol(a, 5) + f + e + k + w[i];
      e = d; d = c; c = rol(b, 30); b = a; a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
  }
  std::vector<uint8_t> out;
  for (uint32_t v : h) for (int s = 24; s >= 0; s -= 8) out.push_back((uint8_t)(v >> s));
  return out;
}

std::vector<uint8_t> sha256(const uint8_t* m, size_t n, bool is224) {
  static const uint32_t K[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01,
      0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc,
      0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
      0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08,
      0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
      0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  if (is224) {
    const uint32_t h224[8] = {0xc1059ed8, 0x367cd507, 0x3070dd17, 0xf70e5939, 0xffc00b31, 0x68581511, 0x64f98fa7, 0xbefa4fa4};
    std::copy(h224, h224 + 8, h);
  }
  const std::vector<uint8_t> p = md_pad(m, n, 64, 8);
  for (size_t o = 0; o < p.size(); o += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[o + 4 * i] << 24 | p[o + 4 * i + 1] << 16 | p[o + 4 * i + 2] << 8 | p[o + 4 * i + 3];
    for (int i = 16; i < 64; i++) {
      const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  std::vector<uint8_t> out;
  for (int i = 0; i < (is224 ? 7 : 8); i++) for (int s = 24; s >= 0; s -= 8) out.push_back((uint8_t)(h[i] >> s));
  return out;
}

std::vector<uint8_t> sha512(const uint8_t* m, size_t n, bool is384) {
  static const uint64_t K[80] = {
      0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull,
      0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull, 0x12835b0145706fbeull,
      0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull, 0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
      0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
      0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull, 0x983e5152ee66dfabull,
      0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
      0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull,
      0x53380d139d95b3dfull, 0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
      0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
      0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull, 0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull,
      0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull,
      0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
      0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull, 0xca273eceea26619cull,
      0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull,
      0x113f9804bef90daeull, 0x1b710b35131c471bull, 0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
      0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
  uint64_t h[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
                   0x510e527fade682d1ull, 0x9b05688c2b3e6c1full, 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
  if (is384) {
    const uint64_t h384[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull, 0x152fecd8f70e5939ull,
                              0x67332667ffc00b31ull, 0x8eb44a8768581511ull, 0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};
    std::copy(h384, h384 + 8, h);
  }
  const std::vector<uint8_t> p = md_pad(m, n, 128, 16);
  for (size_t o = 0; o < p.size(); o += 128) {
    uint64_t w[80];
    for (int i = 0; i < 16; i++) {
      w[i] = 0;
      for (int j = 0; j < 8; j++) w[i] = w[i] << 8 | p[o + 8 * i + j];
    }
    for (int i = 16; i < 80; i++) {
      const uint64_t s0 = ror64(w[i - 15], 1) ^ ror64(w[i - 15], 8) ^ (w[i - 15] >> 7);
      const uint64_t s1 = ror64(w[i - 2], 19) ^ ror64(w[i - 2], 61) ^ (w[i - 2] >> 6);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 80; i++) {
      const uint64_t t1 = hh + (ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      const uint64_t t2 = (ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  std::vector<uint8_t> out;
  for (int i = 0; i < (is384 ? 6 : 8); i++) for (int s = 56; s >= 0; s -= 8) out.push_back((uint8_t)(h[i] >> s));
  return out;
}

std::vector<uint8_t> compute_hash(int out_len, const std::vector<uint8_t>& in) {
  switch (out_len) {
    case 20: return sha1(in.data(), in.size());
    case 28: return sha256(in.data(), in.size(), true);
    case 32: return sha256(in.data(), in.size(), false);
    case 48: return sha512(in.data(), in.size(), true);
    case 64: return sha512(in.data(), in.size(), false);
  }
  fail("Invalid hash output length. Use 20, 28, 32, 48, or 64 bytes.");  // computeHash :101-105
}

// ------------------------------------------------------------------------------------ strings
const char* HEXU = "0123456789ABCDEF";
const char* HEXL = "0123456789abcdef";
std::string hex_of(const uint8_t* b, size_t n, bool upper) {
  std::string s(2 * n, '0');
  const char* d = upper ? HEXU : HEXL;
  for (size_t i = 0; i < n; i++) { s[2 * i] = d[b[i] >> 4]; s[2 * i + 1] = d[b[i] & 15]; }
  return s;
}
std::string lower(std::string s) { for (char& c : s) c = (char)std::tolower((unsigned char)c); return s; }
std::string upper(std::string s) { for (char& c : s) c = (char)std::toupper((unsigned char)c); return s; }
int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
// hexStringToBytes (:246-257) / padding's parse (:21-25): whitespace removed, parseInt per digit pair
std::vector<uint8_t> hex_bytes(const std::string& h0) {
  std::string h;
  for (char c : h0) if (!std::isspace((unsigned char)c)) h.push_back(c);
  std::vector<uint8_t> out;
  for (size_t i = 0; i < h.size(); i += 2) {
    const int a = hexval(h[i]), b = i + 1 < h.size() ? hexval(h[i + 1]) : -1;
    if (a < 0 || (i + 1 < h.size() && b < 0)) fail("non-hex digits in a hex field");
    out.push_back((uint8_t)(b < 0 ? a : a * 16 + b));
  }
  return out;
}
// "<haystack>".split(needle)[0].length: position of the first match, or the whole length
size_t split0(const std::string& hay, const std::string& needle) {
  if (needle.empty()) return 0;
  const size_t p = hay.find(needle);
  return p == std::string::npos ? hay.size() : p;
}

// magnitude bytes (big-endian) -> lowercase hex without leading zeros (BigInt(...).toString(16))
std::string mag_hex(const std::vector<uint8_t>& m) {
  std::string s = hex_of(m.data(), m.size(), false);
  const size_t nz = s.find_first_not_of('0');
  return nz == std::string::npos ? "0" : s.substr(nz);
}
// BigInt("0b" + bits).toString(16)
std::string bits_hex(const std::string& bits) {
  if (bits.empty()) fail("empty bit string in a key");  // BigInt("0b") throws
  std::vector<uint8_t> m((bits.size() + 7) / 8, 0);
  const size_t off = m.size() * 8 - bits.size();
  for (size_t i = 0; i < bits.size(); i++)
    if (bits[i] == '1') m[(off + i) / 8] |= (uint8_t)(0x80 >> ((off + i) % 8));
  return mag_hex(m);
}
// big-endian magnitude -> decimal string
std::string mag_dec(std::vector<uint8_t> m) {
  std::string out;
  size_t i0 = 0;
  while (i0 < m.size() && m[i0] == 0) i0++;
  if (i0 == m.size()) return "0";
  std::vector<uint32_t> parts;  // base 1e9, little-endian
  while (i0 < m.size()) {
    uint64_t r = 0;
    for (size_t i = i0; i < m.size(); i++) {
      const uint64_t cur = (r << 8) | m[i];
      m[i] = (uint8_t)(cur / 1000000000ull);
      r = cur % 1000000000ull;
    }
    parts.push_back((uint32_t)r);
    while (i0 < m.size() && m[i0] == 0) i0++;
  }
  out = std::to_string(parts.back());
  for (size_t k = parts.size() - 1; k-- > 0;) {
    std::string p = std::to_string(parts[k]);
    out += std::string(9 - p.size(), '0') + p;
  }
  return out;
}

// ------------------------------------------------------------------------------------ asn1.js
// reTimeS / reTimeL (asn1.js:2963-2964): [YY]YY MM DD HH [mm [ss [.fff]]] [Z | (+|-)hh [mm]], matched left to
// right (no digit can start what follows an optional digit group, so the greedy match is the regex's)
bool time_ok(const std::string& s, bool long_year) {
  size_t i = 0;
  auto dig = [&](size_t k) { return k < s.size() && s[k] >= '0' && s[k] <= '9'; };
  auto two = [&](const char* lo, const char* hi) {  // two digits within [lo, hi] as a string range
    if (!dig(i) || !dig(i + 1)) return false;
    const std::string v = s.substr(i, 2);
    if (v < lo || v > hi) return false;
    i += 2;
    return true;
  };
  for (int k = 0; k < (long_year ? 4 : 2); k++, i++) if (!dig(i)) return false;
  if (!two("01", "12") || !two("01", "31") || !two("00", "23")) return false;
  if (two("00", "59") && two("00", "59") && i < s.size() && (s[i] == '.' || s[i] == ',') && dig(i + 1)) {
    i++;
    for (int k = 0; k < 3 && dig(i); k++) i++;
  }
  if (i < s.size() && s[i] == 'Z') i++;
  else if (i < s.size() && (s[i] == '+' || s[i] == '-')) {
    const bool plus = s[i] == '+';
    i++;
    if (!two("00", plus ? "14" : "12")) return false;
    two("00", "59");
  }
  return i == s.size();
}

struct Node {
  int64_t start;    // stream.pos of the element
  int64_t header;   // tag + length bytes
  int64_t len;      // content length (negative: undefined-length content, as asn1.js stores it)
  int tclass;
  bool cons;
  uint64_t tnum;
  bool has_sub = false;
  std::vector<int> sub;
};

// Named curves: the "d" entries of asn1.js's OID table (:238-2958) that an ECDSA key can name
struct OidName { const char* oid; const char* d; };
const OidName CURVE_NAMES[] = {
    {"1.2.840.10045.3.1.1", "prime192v1"}, {"1.2.840.10045.3.1.7", "prime256v1"}, {"1.3.132.0.33", "secp224r1"},
    {"1.3.132.0.34", "secp384r1"}, {"1.3.132.0.35", "secp521r1"}, {"1.3.36.3.3.2.8.1.1.1", "brainpoolP160r1"},
    {"1.3.36.3.3.2.8.1.1.3", "brainpoolP192r1"}, {"1.3.36.3.3.2.8.1.1.5", "brainpoolP224r1"},
    {"1.3.36.3.3.2.8.1.1.7", "brainpoolP256r1"}, {"1.3.36.3.3.2.8.1.1.9", "brainpoolP320r1"},
    {"1.3.36.3.3.2.8.1.1.11", "brainpoolP384r1"}, {"1.3.36.3.3.2.8.1.1.13", "brainpoolP512r1"}};

struct Tree {
  const uint8_t* b;
  int64_t n;
  std::vector<Node> nodes;
  int root = -1;

  Tree(const uint8_t* p, size_t len) : b(p), n((int64_t)len) {
    int64_t pos = 0;
    root = decode(pos);
    if (root < 0) fail(err);
    for (size_t i = 0; i < nodes.size(); i++) {  // simplifyASN1 calls content() and toHexString() on every node
      if (!content_ok((int)i)) fail("content() throws on an element");
      const Node& x = nodes[i];
      if (x.start + x.header + (x.len < 0 ? -x.len : x.len) > n) fail("element past the end of the stream");
    }
  }
  uint8_t get(int64_t pos) const {  // Stream.get (:3028-3034)
    if (pos < 0 || pos >= n) fail("Requesting byte offset " + std::to_string(pos) + " on a stream of length " + std::to_string(n));
    return b[pos];
  }
  const Node& at(int i) const { return nodes[i]; }
  int64_t content_pos(const Node& x) const { return x.start + x.header; }
  bool universal(const Node& x) const { return x.tclass == 0; }
  bool is_eoc(const Node& x) const { return x.tclass == 0 && x.tnum == 0; }

  // ASN1.decode (:3520-3589). Returns the node index, or -1 where asn1.js throws (err says why): the
  // encapsulation attempts fail often, so failure is a return value here, not a C++ exception
  // (whose unwinding serialises the host threads of a bulk call)
  std::string err;
  bool byte(int64_t p, uint8_t& v) const {
    if (p < 0 || p >= n) return false;
    v = b[p];
    return true;
  }
  int bad(const char* why) { err = why; return -1; }
  // Nesting cap: the input is untrusted DER, and every walk over the tree (decode, content_ok, the key
  // and digest searches) recurses per level. asn1.js has no cap of its own (it throws a RangeError when
  // the JS stack runs out); real EF.SOD files nest < 20 levels, so anything past 64 is rejected here
  // instead of overflowing a host thread's stack.
  static constexpr int MAX_DEPTH = 64;
  int decode(int64_t& pos, int depth = 0) {
    if (depth > MAX_DEPTH) return bad("ASN.1 nesting deeper than 64 levels");
    Node x{};
    x.start = pos;
    uint8_t t;
    if (!byte(pos++, t)) return bad("Requesting byte offset past the end of the stream");
    x.tclass = t >> 6;
    x.cons = (t & 0x20) != 0;
    x.tnum = t & 0x1F;
    if (x.tnum == 0x1F) {  // long tag
      uint64_t v = 0;
      do {
        if (!byte(pos++, t)) return bad("Requesting byte offset past the end of the stream");
        v = v * 128 + (t & 0x7F);
      } while (t & 0x80);
      x.tnum = v;
    }
    // decodeLength (:3506-3519)
    uint8_t lb;
    if (!byte(pos++, lb)) return bad("Requesting byte offset past the end of the stream");
    int64_t len;
    bool undef = false;
    if ((lb & 0x7F) == lb) len = lb;
    else if ((lb & 0x7F) == 0) { undef = true; len = 0; }
    else {
      const int k = lb & 0x7F;
      if (k > 6) return bad("Length over 48 bits not supported");
      len = 0;
      for (int i = 0; i < k; i++) {
        uint8_t d;
        if (!byte(pos++, d)) return bad("Requesting byte offset past the end of the stream");
        len = len * 256 + d;
      }
    }
    const int64_t start = pos;
    x.header = start - x.start;
    const size_t mark = nodes.size();
    std::vector<int> sub;
    auto get_sub = [&]() -> bool {
      sub.clear();
      if (!undef) {
        const int64_t end = start + len;
        if (end > n) { err = "Container has a length past the end of the stream"; return false; }
        while (pos < end) {
          const int s = decode(pos, depth + 1);
          if (s < 0) return false;
          sub.push_back(s);
        }
        if (pos != end) { err = "Content size is not correct for container"; return false; }
      } else {
        for (;;) {
          const int s = decode(pos, depth + 1);
          if (s < 0) return false;
          if (is_eoc(nodes[s])) break;
          sub.push_back(s);
        }
        len = start - pos;
        undef = false;
      }
      return true;
    };
    bool has_sub = false;
    if (x.cons) {
      if (!get_sub()) return -1;
      has_sub = true;
    } else if (x.tclass == 0 && (x.tnum == 0x03 || x.tnum == 0x04)) {  // encapsulation attempt (:3561-3582)
      const bool was_undef = undef;
      const int64_t len0 = len;
      uint8_t ub = 0;
      bool ok = x.tnum != 0x03 || (byte(pos++, ub) && ub == 0);
      ok = ok && get_sub();
      for (size_t k = 0; ok && k < sub.size(); k++) ok = !is_eoc(nodes[sub[k]]) && content_ok(sub[k]);
      if (ok) has_sub = true;
      else {  // silently ignored: a plain string
        nodes.resize(mark);
        sub.clear();
        if (was_undef) { undef = true; len = len0; }
      }
    }
    if (!has_sub) {
      if (undef) return bad("We can't skip over an invalid tag with undefined length");
      pos = start + (len < 0 ? -len : len);
    }
    x.len = len;
    x.has_sub = has_sub;
    x.sub = std::move(sub);
    nodes.push_back(std::move(x));
    return (int)nodes.size() - 1;
  }

  // where content() (:3387-3450) and the parsers it calls throw
  bool utf8_ok(int64_t s, int64_t e) const {  // parseStringUTF (:3117-3147)
    auto ex = [&](int64_t i) { uint8_t c; return byte(i, c) && c >= 0x80 && c < 0xC0; };
    for (int64_t i = s; i < e;) {
      uint8_t c;
      if (!byte(i++, c)) return false;
      if (c < 0x80) continue;
      if (c < 0xC0) return false;
      if (c < 0xE0) { if (!ex(i++)) return false; continue; }
      if (c < 0xF0) { if (!ex(i) || !ex(i + 1)) return false; i += 2; continue; }
      if (c < 0xF8) {
        if (!ex(i) || !ex(i + 1) || !ex(i + 2)) return false;
        const uint32_t cp = ((uint32_t)(c & 7) << 18) | ((uint32_t)(b[i] & 0x3F) << 12) | ((uint32_t)(b[i + 1] & 0x3F) << 6) |
                            (b[i + 2] & 0x3F);
        i += 3;
        if (cp < 0x10000) return false;  // surrogate(): overlong
        continue;
      }
      return false;
    }
    return true;
  }
  // recurse (:3294-3312): constructed strings made of same-tag pieces are read piecewise
  bool piecewise(const Node& x) const {
    if (!(x.cons && x.has_sub)) return false;
    for (int s : x.sub)
      if (nodes[s].tclass != x.tclass || nodes[s].tnum != x.tnum) return false;
    return true;
  }
  bool content_ok(int i) const {
    const Node& x = nodes[i];
    const int64_t c = content_pos(x), len = x.len < 0 ? -x.len : x.len;
    uint8_t v;
    if (!universal(x)) return true;  // "(n elem)" or parseOctetString: no throw
    auto pieces = [&]() { for (int s : x.sub) if (!content_ok(s)) return false; return true; };
    switch (x.tnum) {
      case 0x01: case 0x02: case 0x0A: return byte(c, v);  // BOOLEAN / INTEGER / ENUMERATED read their first byte
      case 0x03:                                           // BIT_STRING
        if (piecewise(x)) return pieces();
        return byte(c, v) && v <= 7;
      case 0x0C:                                           // UTF8String
        if (piecewise(x)) return pieces();
        return utf8_ok(c, c + len);
      case 0x14:                                           // TeletexString: a diacritic reads the next byte
        if (piecewise(x)) return pieces();
        for (int64_t k = c; k < c + len; ++k) {
          if (!byte(k, v)) return false;
          if (v >= 0xC0 && v <= 0xCF && !byte(++k, v)) return false;
        }
        return true;
      case 0x1E:                                           // BMPString: byte pairs
        if (piecewise(x)) return pieces();
        for (int64_t k = c; k < c + len; k += 2)
          if (!byte(k, v) || !byte(k + 1, v)) return false;
        return true;
      case 0x17: case 0x18: {                              // UTCTime / GeneralizedTime (parseTime :3157-3183)
        std::string s;
        for (int64_t k = c; k < c + len; k++) {
          if (!byte(k, v)) return false;
          s.push_back((char)v);
        }
        return time_ok(s, x.tnum == 0x18);
      }
      default: return true;
    }
  }

  // content() strings for the element types the extractors read
  std::string octets_str(const Node& x) const {  // parseOctetString (:3229-3248) via recurse
    if (piecewise(x)) {
      std::string s;
      for (int k : x.sub) s += octets_str(nodes[k]);
      return s;
    }
    const int64_t c = content_pos(x), len = x.len < 0 ? -x.len : x.len;
    bool printable = utf8_ok(c, c + len);
    for (int64_t i = c; printable && i < c + len;) {  // code units, for checkPrintable (:2992-2999)
      const uint8_t ch = b[i++];
      uint32_t cp;
      if (ch < 0x80) cp = ch;
      else if (ch < 0xE0) { cp = ((uint32_t)(ch & 0x1F) << 6) | (b[i] & 0x3F); i += 1; }
      else if (ch < 0xF0) { cp = ((uint32_t)(ch & 0x0F) << 12) | ((uint32_t)(b[i] & 0x3F) << 6) | (b[i + 1] & 0x3F); i += 2; }
      else { cp = 0x10000; i += 3; }
      if (cp < 32 && cp != 9 && cp != 10 && cp != 13) printable = false;
    }
    if (printable) {  // the text itself (UTF-8 bytes), not hex
      std::string s;
      for (int64_t i = c; i < c + len; i++) s.push_back((char)b[i]);
      return s;
    }
    return hex_of(b + c, (size_t)len, true);
  }
  std::string bits_str(const Node& x) const {  // parseBitString (:3213-3228) via recurse
    if (piecewise(x)) {
      std::string s;
      for (int k : x.sub) s += bits_str(nodes[k]);
      return s;
    }
    const int64_t c = content_pos(x), len = x.len < 0 ? -x.len : x.len;
    const int unused = get(c);
    std::string s(len > 1 ? (size_t)(8 * (len - 1)) : 0, '0');
    size_t o = 0;
    for (int64_t i = c + 1; i < c + len; i++) {
      const int skip = i == c + len - 1 ? unused : 0;
      for (int j = 7; j >= skip; --j) s[o++] = ((b[i] >> j) & 1) ? '1' : '0';
    }
    s.resize(o);
    return s;
  }
  // parseInteger (:3184-3212) as a magnitude; negative integers are outside what the walks expect
  std::vector<uint8_t> integer_mag(const Node& x) const {
    const int64_t c = content_pos(x), len = x.len < 0 ? -x.len : x.len;
    if (len == 0 || (get(c) & 0x80)) fail("negative or empty INTEGER where the reference reads a magnitude");
    return std::vector<uint8_t>(b + c, b + c + len);
  }
  std::string oid_str(const Node& x) const {  // parseOID (:3249-3288), the curve-name part of the table only
    const int64_t c = content_pos(x), len = x.len < 0 ? -x.len : x.len;
    std::string s;
    uint64_t v = 0;
    bool first = true;
    for (int64_t i = c; i < c + len; i++) {
      v = v * 128 + (b[i] & 0x7F);
      if (!(b[i] & 0x80)) {
        if (first) {
          const uint64_t m = v < 80 ? (v < 40 ? 0 : 1) : 2;
          s = std::to_string(m) + "." + std::to_string(v - 40 * m);
          first = false;
        } else {
          s += "." + std::to_string(v);
        }
        v = 0;
      }
    }
    for (const OidName& o : CURVE_NAMES)
      if (s == o.oid) return s + "\n" + o.d;
    return s;
  }
  std::string name(const Node& x) const {  // typeName (:3347-3385) for the names the walks compare
    if (x.tclass == 2) return "[" + std::to_string(x.tnum) + "]";
    if (x.tclass != 0) return "other";
    switch (x.tnum) {
      case 0x02: return "INTEGER";
      case 0x03: return "BIT_STRING";
      case 0x04: return "OCTET_STRING";
      case 0x06: return "OBJECT_IDENTIFIER";
      case 0x10: return "SEQUENCE";
      case 0x11: return "SET";
    }
    return "universal";
  }
  // content() as the salt check reads it: null (falsy) or the string
  bool content_any(const Node& x, std::string& s) const {
    if (!universal(x)) {
      if (x.has_sub) { s = "(" + std::to_string(x.sub.size()) + " elem)"; return true; }
      s = octets_str(x);
      return true;
    }
    switch (x.tnum) {
      case 0x01: s = b[content_pos(x)] ? "true" : "false"; return true;
      case 0x02: case 0x0A: {
        const int64_t c = content_pos(x), len = x.len < 0 ? -x.len : x.len;
        if (len > 0 && (b[c] & 0x80)) { s = "-"; return true; }  // negative: a non-numeric salt either way
        s = mag_dec(std::vector<uint8_t>(b + c, b + c + len));
        return true;
      }
      case 0x03: s = bits_str(x); return true;
      case 0x04: s = octets_str(x); return true;
      case 0x06: s = oid_str(x); return true;
      case 0x10: case 0x11: s = x.has_sub ? "(" + std::to_string(x.sub.size()) + " elem)" : "(no elem)"; return true;
      case 0x05: return false;
    }
    s = "?";
    return true;
  }
  std::string dump(const Node& x) const {  // toHexString('raw'): the whole element, upper-case hex
    const int64_t e = x.start + x.header + (x.len < 0 ? -x.len : x.len);
    for (int64_t k = x.start; k < e; k++) get(k);
    return hex_of(b + x.start, (size_t)(e - x.start), true);
  }
  const Node& sub(const Node& x, long k) const {  // x.sub[k] / x.sub.slice(k)[0] (k < 0 from the end)
    if (!x.has_sub) fail("element has no sub-elements");
    const long m = (long)x.sub.size();
    const long i = k < 0 ? m + k : k;
    if (i < 0 || i >= m) fail("sub-element index out of range");
    return nodes[x.sub[i]];
  }
};

// getFirstOctetString (:269-284)
const Node* first_octets(const Tree& T, const Node& x) {
  if (T.name(x) == "OCTET_STRING") return &x;
  if (x.has_sub)
    for (int s : x.sub)
      if (const Node* r = first_octets(T, T.nodes[s])) return r;
  return nullptr;
}
// getZero (:322-358): the [0] whose last element is SEQUENCE { OID, SET { OCTET STRING } }
const Node* get_zero(const Tree& T, const Node& x) {
  if (T.name(x) == "[0]" && x.has_sub && !x.sub.empty()) {
    const Node& last = T.nodes[x.sub.back()];
    if (T.name(last) == "SEQUENCE" && last.has_sub && last.sub.size() == 2 && T.name(T.nodes[last.sub[0]]) == "OBJECT_IDENTIFIER") {
      const Node& st = T.nodes[last.sub[1]];
      if (T.name(st) == "SET" && st.has_sub && st.sub.size() == 1 && T.name(T.nodes[st.sub[0]]) == "OCTET_STRING") return &x;
    }
  }
  if (x.has_sub)
    for (int s : x.sub)
      if (const Node* r = get_zero(T, T.nodes[s])) return r;
  return nullptr;
}
// findParentOfLastOctetString (:387-412)
void last_octets(const Tree& T, const Node& x, const Node* parent, const Node*& res, const Node*& par) {
  if (T.name(x) == "OCTET_STRING") { res = &x; par = parent; }
  if (x.has_sub)
    for (int s : x.sub) {
      const Node *r = nullptr, *p = nullptr;
      last_octets(T, T.nodes[s], &x, r, p);
      if (r) { res = r; par = p; }
    }
}
// get_ecdsa_key_location (:414-437)
const Node* ecdsa_key_loc(const Tree& T, const Node& x) {
  if (x.has_sub && x.sub.size() >= 2) {
    const Node& second = T.nodes[x.sub[1]];
    if (T.name(second) == "BIT_STRING" && T.bits_str(second).rfind("00000100", 0) == 0) return &x;
  }
  if (x.has_sub)
    for (int s : x.sub)
      if (const Node* r = ecdsa_key_loc(T, T.nodes[s])) return r;
  return nullptr;
}
// get_rsa_key_location (:455-481)
const Node* rsa_key_loc(const Tree& T, const Node& x) {
  if (T.name(x) == "BIT_STRING" && x.has_sub)
    for (int s : x.sub) {
      const Node& c = T.nodes[s];
      if (T.name(c) == "SEQUENCE" && c.has_sub && c.sub.size() == 2 && T.name(T.nodes[c.sub[0]]) == "INTEGER" &&
          T.name(T.nodes[c.sub[1]]) == "INTEGER")
        return &x;
    }
  if (x.has_sub)
    for (int s : x.sub)
      if (const Node* r = rsa_key_loc(T, T.nodes[s])) return r;
  return nullptr;
}

// padding (:11-91) + processPassport's bit conversion (:701-757): BigInt(padded).toString(2), then
// zeros prepended up to a multiple of the block
std::vector<uint8_t> padded_bits(const std::vector<uint8_t>& msg, int block_bits) {
  const std::vector<uint8_t> p = md_pad(msg.data(), msg.size(), block_bits / 8, block_bits == 512 ? 8 : 16);
  size_t nz = 0;  // leading zero bits, dropped by the BigInt round trip
  while (nz < p.size() * 8 && !((p[nz / 8] >> (7 - nz % 8)) & 1)) nz++;
  const size_t sig = std::max<size_t>(p.size() * 8 - nz, 1);  // BigInt 0 -> "0"
  const size_t total = sig % block_bits ? (sig / block_bits + 1) * block_bits : sig;
  std::vector<uint8_t> out(total, 0);
  for (size_t i = 0, o = total - (p.size() * 8 - nz); i < p.size() * 8 - nz; i++, o++) {
    const size_t k = nz + i;
    out[o] = (p[k / 8] >> (7 - k % 8)) & 1;
  }
  return out;
}

// bigintToArray(n, k, x) (:113-123) over a hex value: k limbs of n bits, low first, as 9-byte little-endian
// buffers (room for the 66-bit limbs of fields wider than 512 bits); bits above n * k are dropped
std::vector<std::array<uint8_t, 9>> to_limbs(const std::string& hex, int nbits, int k) {
  std::vector<uint8_t> le((hex.size() + 1) / 2 + 10, 0);  // little-endian bytes of the value
  for (size_t i = 0; i < hex.size(); i++) {
    const int v = hexval(hex[hex.size() - 1 - i]);
    if (v < 0) fail("non-hex key or signature value");
    le[i / 2] |= (uint8_t)(v << (4 * (i & 1)));
  }
  std::vector<std::array<uint8_t, 9>> out(k);
  for (int l = 0; l < k; l++) {
    out[l].fill(0);
    const size_t bit0 = (size_t)l * nbits;
    for (int j = 0; j < nbits; j += 8) {  // byte j / 8 of the limb = bits [bit0 + j, bit0 + j + 8)
      const size_t bi = bit0 + j, byte = bi / 8, sh = bi % 8;
      unsigned v = byte < le.size() ? le[byte] >> sh : 0;
      if (sh && byte + 1 < le.size()) v |= (unsigned)le[byte + 1] << (8 - sh);
      const int keep = std::min(8, nbits - j);
      out[l][j / 8] = (uint8_t)(v & ((1u << keep) - 1));
    }
  }
  return out;
}

struct Parsed {
  pzk_passport_info info{};
  std::vector<uint8_t> dg1_bits, dg15_bits, ec_bits, sa_bits;
  std::vector<std::array<uint8_t, 9>> pk_limbs, sig_limbs;
};

int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// processPassport (:674-816) without the file I/O; returns the arrays writeToJson writes
Parsed process(const pzk_passport_src& src) {
  Parsed P;
  pzk_passport_info& I = P.info;
  const std::vector<uint8_t> dg1(src.dg1, src.dg1 + src.dg1_len), dg15(src.dg15, src.dg15 + src.dg15_len);
  const Tree T(src.sod, src.sod_len);
  const Node& root = T.nodes[T.root];
  // extract_encapsulated_content (:286-292)
  const Node* ec = first_octets(T, root);
  if (!ec) fail("no OCTET STRING in the SOD");
  const Node& dgh = T.sub(T.sub(T.sub(T.sub(*ec, 0), 2), 0), 1);
  const int dg_hash_type = (int)(dgh.len < 0 ? -dgh.len : dgh.len);
  const std::string ec_hex = T.octets_str(*ec);
  // extract_signed_atributes (:360-366)
  const Node* sa = get_zero(T, root);
  if (!sa) fail("no signed attributes ([0] ending in a messageDigest-shaped attribute)");
  const Node& mdn = T.sub(T.sub(T.sub(*sa, -1), -1), 0);
  const int hash_type = (int)(mdn.len < 0 ? -mdn.len : mdn.len);
  const std::string sa_dump = T.dump(*sa);
  const std::string sa_hex = "31" + sa_dump.substr(2);
  const int dg_block = dg_hash_type <= 32 ? 512 : 1024, hash_block = hash_type <= 32 ? 512 : 1024;
  const std::vector<uint8_t> ec_bytes = hex_bytes(ec_hex), sa_bytes = hex_bytes(sa_hex);
  P.dg1_bits = padded_bits(dg1, dg_block);
  if (!dg15.empty()) P.dg15_bits = padded_bits(dg15, dg_block);
  P.ec_bits = padded_bits(ec_bytes, hash_block);
  P.sa_bits = padded_bits(sa_bytes, hash_block);
  // extract_signature (:368-385)
  const Node *oct = nullptr, *parent = nullptr;
  last_octets(T, root, nullptr, oct, parent);
  if (!oct || !parent) fail("no signature OCTET STRING");
  std::string salt_s;
  bool salt_truthy = false;
  {
    const Node& params = T.sub(T.sub(*parent, -2), -1);
    if (params.has_sub) {  // ...sub?.slice(-1)[0].sub[0].content
      const Node& last = T.sub(params, -1);
      std::string s;
      if (T.content_any(T.sub(last, 0), s) && !s.empty()) { salt_s = s; salt_truthy = true; }
    }
  }
  const bool ecdsa_sig = oct->has_sub;
  std::string sig_r, sig_s, sig_n;
  if (ecdsa_sig) {
    const Node& rs = T.sub(*oct, 0);
    sig_r = mag_hex(T.integer_mag(T.sub(rs, 0)));
    sig_s = mag_hex(T.integer_mag(T.sub(rs, 1)));
  } else {
    sig_n = T.octets_str(*oct);
  }
  // public key (:760-763): sig.salt || sig.salt == 0 holds for every RSA-shaped signature ({n, salt}) and
  // for no ECDSA one ({r, s}: salt undefined)
  const bool salt_zero_like = !salt_truthy || salt_s == "0";  // sig.salt == 0 (loose)
  std::string pk_n, pk_exp, pk_x, pk_y, pk_param;
  bool pk_is_ec = false, has_param = false;
  if (!ecdsa_sig) {
    const Node* loc = rsa_key_loc(T, root);  // extract_rsa_pubkey (:483-490)
    if (!loc) fail("no RSA public key in the SOD");
    pk_n = mag_hex(T.integer_mag(T.sub(T.sub(*loc, 0), 0)));
    pk_exp = mag_hex(T.integer_mag(T.sub(T.sub(*loc, 0), 1)));
  } else {
    const Node* loc = ecdsa_key_loc(T, root);  // extract_ecdsa_pubkey (:439-453)
    if (!loc) fail("no EC public key in the SOD");
    const std::string bits = T.bits_str(T.sub(*loc, 1)).substr(8);
    pk_x = bits_hex(bits.substr(0, bits.size() / 2));
    pk_y = bits_hex(bits.substr(bits.size() / 2));
    const Node& p1 = T.sub(T.sub(*loc, 0), 1);
    if (p1.has_sub) pk_param = T.octets_str(T.sub(T.sub(p1, 2), 0));
    else {  // named curve: content().split("\n")[1]
      std::string o;
      if (!T.content_any(p1, o)) fail("null content where the reference splits the curve name");
      const size_t nl = o.find('\n');
      if (nl != std::string::npos) pk_param = o.substr(nl + 1, o.find('\n', nl + 1) - nl - 1);
    }
    has_param = !pk_param.empty();
    pk_is_ec = true;
  }
  // getSigType (:157-244)
  int sig_type = 0;
  if (salt_truthy && !pk_is_ec) {
    const size_t L = pk_n.size();
    if (L == 512 && pk_exp == "3" && salt_s == "32" && hash_type == 32) sig_type = 10;
    else if (L == 512 && pk_exp == "10001" && salt_s == "32" && hash_type == 32) sig_type = 11;
    else if (L == 512 && pk_exp == "10001" && salt_s == "64" && hash_type == 32) sig_type = 12;
    else if (L == 512 && pk_exp == "10001" && salt_s == "48" && hash_type == 48) sig_type = 13;
    else if (L == 768 && pk_exp == "10001" && salt_s == "32" && hash_type == 32) sig_type = 14;
  }
  if (!sig_type && salt_zero_like && !pk_is_ec && !ecdsa_sig) {
    const size_t L = pk_n.size();
    if (L == 512 && pk_exp == "10001" && hash_type == 32) sig_type = 1;
    else if (L == 1024 && pk_exp == "10001" && hash_type == 32) sig_type = 2;
    else if (L == 512 && pk_exp == "10001" && hash_type == 20) sig_type = 3;
  }
  if (!sig_type && ecdsa_sig) {
    if (pk_param == "7D5A0975FC2C3057EEF67530417AFFE7FB8055C126DC5C6CE94A4B44F330B5D9") sig_type = 21;
    else if (pk_param == "FFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFC") sig_type = 20;
    else if (pk_param == "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFE") sig_type = 24;
    else if (pk_param == "7BC382C63D8C150C3C72080ACE05AFA0C2BEA28E4FB22787139165EFBA91F90F8AA5814A503AD4EB04A8C7DD22CE2826")
      sig_type = 25;
    else if (pk_param == "7830A3318B603B89E2327145AC234CC594CBDD8D3DF91610A83441CAEA9863BC2DED5D5AA8253AA10A2EF1C98B9AC8B57F"
                         "1117A72BF2C7B9E7C1AC4D77FC94CA")
      sig_type = 26;
    else if (pk_param == "secp521r1") sig_type = 27;
  }
  // shifts (:767-772): position of the hex digest in the hex text, in bytes (x8 -> bits)
  auto hash_hex = [&](int len, const std::vector<uint8_t>& m) { const auto h = compute_hash(len, m); return hex_of(h.data(), h.size(), false); };
  const std::string ec_lc = lower(ec_hex);
  const long dg1_nib = (long)split0(ec_lc, hash_hex(dg_hash_type, dg1));
  const long ec_nib = (long)split0(lower(sa_dump), hash_hex(hash_type, ec_bytes));
  const long dg15_nib = dg15.empty() ? 0 : (long)split0(ec_lc, hash_hex(dg_hash_type, dg15));
  // extractFromDg15 (:492-571)
  int aa_sig = 0;
  long aa_nib = 0;
  if (!dg15.empty()) {
    const Tree D(dg15.data(), dg15.size());
    const Node& d0 = D.nodes[D.root];
    const Node& spki = D.sub(d0, 0);
    std::string kb;
    if (!D.content_any(D.sub(spki, 1), kb)) fail("null content where the reference slices the DG15 key bits");
    const std::string dd = D.dump(d0);
    if (kb.substr(0, 8) == "00000100") {
      const std::string pkb = kb.substr(8);
      const std::string p = upper(mag_hex(D.integer_mag(D.sub(D.sub(D.sub(spki, 0), 1), 4))));
      if (p == "A9FB57DBA1EEA9BC3E660A909D838D718C397AA3B561A6F7901E0E82974856A7") aa_sig = 21;
      else if (p == "FFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF") aa_sig = 20;
      else if (p == "D35E472036BC4FB7E13C785ED201E065F98FCFA6F6F40DEF4F92B9EC7893EC28FCD412B1F1B32E27") aa_sig = 22;
      else if (p == "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFFFFFFFFFFFF") aa_sig = 23;
      else fail("unknown tech! (DG15 EC key on an unlisted curve)", PZK_PP_UNKNOWN);
      aa_nib = (long)split0(dd, upper(bits_hex(pkb.substr(0, pkb.size() / 2))));
    } else {
      const Node& loc = D.sub(D.sub(spki, 1), 0);
      aa_sig = 1;
      aa_nib = (long)split0(dd, upper(mag_hex(D.integer_mag(D.sub(loc, 0)))));
    }
  }
  // getChunkedParams (:590-626)
  long field = 0;
  bool field_unknown = false;  // "UNKNOWN FIELD SIZE": neither <= 512 nor > 512
  if (has_param) {
    bool allhex = pk_param.size() % 2 == 0;
    for (char ch : pk_param) allhex = allhex && hexval(ch) >= 0;
    if (allhex) field = (long)pk_param.size() * 4;
    else {
      size_t d = pk_param.find_first_of("0123456789");
      if (d == std::string::npos) field_unknown = true;
      else field = std::stol(pk_param.substr(d, pk_param.find_first_not_of("0123456789", d) - d));
    }
  }
  const std::string& kx = pk_is_ec ? pk_x : pk_n;
  const int chunk_number = !field_unknown && field <= 512 ? ceil_div((long)kx.size(), 16) : 8;
  const int chunk_bits = !field_unknown && field > 512 ? 66 : 64;
  if (pk_is_ec) {
    P.pk_limbs = to_limbs(pk_x, chunk_bits, chunk_number);
    const auto py = to_limbs(pk_y, chunk_bits, chunk_number);
    P.pk_limbs.insert(P.pk_limbs.end(), py.begin(), py.end());
    if (!ecdsa_sig) fail("EC key with an RSA-shaped signature");
    P.sig_limbs = to_limbs(sig_r, chunk_bits, chunk_number);
    const auto ss = to_limbs(sig_s, chunk_bits, chunk_number);
    P.sig_limbs.insert(P.sig_limbs.end(), ss.begin(), ss.end());
  } else {
    if (ecdsa_sig) fail("RSA key with an ECDSA-shaped signature");
    P.pk_limbs = to_limbs(pk_n, chunk_bits, chunk_number);
    P.sig_limbs = to_limbs(lower(sig_n), chunk_bits, chunk_number);
  }
  // writeToCircom arguments (:775-800) and the name (:772)
  const int doc = dg1.size() == 93 ? 3 : 1;
  const int ec_blocks = hash_type <= 32 ? ceil_div((long)ec_bytes.size() + 8, 64) : ceil_div((long)ec_bytes.size() + 8, 128);
  const int dg15_blocks = dg15.empty() ? 0 : dg_hash_type <= 32 ? ceil_div((long)dg15.size() + 8, 64) : ceil_div((long)dg15.size() + 8, 128);
  I.params.circuit = PZK_CIRCUIT_REGISTER;
  I.params.signature_type = sig_type;
  I.params.dg_hash_type = dg_hash_type * 8;
  I.params.document_type = doc;
  I.params.ec_block_number = ec_blocks;
  I.params.ec_shift = (int32_t)(ec_nib * 4);
  I.params.dg1_shift = (int32_t)(dg1_nib * 4);
  I.params.aa_signature_algo = aa_sig;
  I.params.dg15_shift = (int32_t)(dg15_nib * 4);
  I.params.dg15_block_number = dg15_blocks;
  I.params.aa_shift = (int32_t)(aa_nib * 4);
  I.ref_aa_shift = (int32_t)(aa_nib / 2);
  I.dg_hash_bytes = dg_hash_type;
  I.hash_bytes = hash_type;
  I.dg1_len = (int32_t)dg1.size();
  I.dg15_len = (int32_t)dg15.size();
  I.ec_len = (int32_t)ec_bytes.size();
  I.sa_len = (int32_t)sa_bytes.size();
  I.chunk_number = chunk_number;
  I.chunk_bits = chunk_bits;
  I.salt = salt_truthy ? std::atoi(salt_s.c_str()) : 0;
  auto times8 = [](long nib) { return std::to_string(nib * 4); };
  std::string name = "registerIdentity_" + std::to_string(sig_type) + "_" + std::to_string(dg_hash_type * 8) + "_" +
                     std::to_string(doc) + "_" + std::to_string(ec_blocks) + "_" + std::to_string(ec_nib * 32) + "_" +
                     std::to_string(dg1_nib * 32) + "_";
  name += dg15.empty() ? std::string("NA")
                       : std::to_string(aa_sig) + "_" + std::to_string(dg15_nib * 32) + "_" + std::to_string(dg15_blocks) + "_" +
                             times8(aa_nib);
  std::snprintf(I.name, sizeof(I.name), "%s", name.c_str());
  return P;  // SIGNATURE_TYPE 0: processPassport prints "UNKNOWN TECHONOLY" (:765) and writes the files anyway

}

void put_bits(uint8_t* row, size_t& o, const std::vector<uint8_t>& bits) {
  for (uint8_t v : bits) { row[32 * o] = v; o++; }
}

}  // namespace

extern "C" int pzk_passport_parse(const pzk_passport_src* src, pzk_passport_info* info) {
  if (!src || !info || !src->sod || (!src->dg1 && src->dg1_len) || (!src->dg15 && src->dg15_len))
    return pzk::api_fail(PZK_E_ARG, "pzk_passport_parse: null argument");
  try {
    *info = process(*src).info;
    return 0;
  } catch (const Fail& e) {
    return pzk::api_fail(PZK_E_ARG, std::string("pzk_passport_parse: ") + e.what());
  } catch (const std::exception& e) {
    return pzk::api_fail(PZK_E_ARG, std::string("pzk_passport_parse: ") + e.what());
  }
}

extern "C" int pzk_passport_inputs(const pzk_params* params, const pzk_passport_src* srcs, size_t n, const uint8_t* identity,
                                   uint8_t* rows, int32_t* status, int threads) {
  if (!params || (n && (!srcs || !rows || !status))) return pzk::api_fail(PZK_E_ARG, "pzk_passport_inputs: null argument");
  if (params->circuit != PZK_CIRCUIT_REGISTER) return pzk::api_fail(PZK_E_PARAMS, "pzk_passport_inputs: not a register instance");
  pzk_info li{};
  uint32_t nreg = 0;
  if (int rc = pzk_layout_query(params, &li, &nreg)) return rc;
  const int sig = params->signature_type;
  // limbs per coordinate: CHUNK_NUMBER of the circuit (registerIdentityBuilder.circom:59-99; 7 x 32 bits for SIG 24,
  // where processPassport's getChunkedParams (:590-626) makes 4 x 64: such rows get PZK_PP_LIMBS)
  const int K = sig == 24 ? 7 : sig == 25 ? 6 : sig >= 20 ? 4 : sig == 2 ? 64 : (sig == 4 || sig == 14) ? 48 : 32;
  const int hb = (sig == 13 || sig == 25) ? 1024 : 512;  // HASH_BLOCK_SIZE (registerIdentityBuilder.circom:104-111)
  const size_t ecL = (size_t)params->ec_block_number * hb, d15L = (size_t)params->dg15_block_number * hb;
  const size_t n_in = 1 + ecL + 1024 + d15L + 1024 + 2 * (size_t)(sig >= 20 ? 2 * K : K) + 80 + 1;
  if (n_in != li.n_inputs) return pzk::api_fail(PZK_E_PARAMS, "pzk_passport_inputs: input layout mismatch");
  const size_t row_bytes = 32 * n_in;
  auto work = [&](size_t i) {
    uint8_t* row = rows + row_bytes * i;
    std::memset(row, 0, row_bytes);
    try {
      const Parsed P = process(srcs[i]);
      if (P.info.params.signature_type == 0) { status[i] = PZK_PP_UNKNOWN; return; }
      pzk_params want = *params, got = P.info.params;
      want.size_arg = got.size_arg = 0;
      if (std::memcmp(&want, &got, sizeof want)) { status[i] = PZK_PP_PARAMS; return; }
      const int coords = sig >= 20 ? 2 : 1;
      if (P.info.chunk_bits != (sig == 24 ? 32 : 64) || P.info.chunk_number != K || (int)P.pk_limbs.size() != coords * K) {
        status[i] = PZK_PP_LIMBS;
        return;
      }
      if (P.ec_bits.size() != ecL || P.dg1_bits.size() != 1024 || P.dg15_bits.size() != d15L || P.sa_bits.size() != 1024) {
        status[i] = PZK_PP_SIZE;
        return;
      }
      const uint8_t* id = identity ? identity + (size_t)82 * 32 * i : nullptr;
      size_t o = 0;
      if (id) std::memcpy(row, id, 32);  // slaveMerkleRoot
      o = 1;
      put_bits(row, o, P.ec_bits);
      put_bits(row, o, P.dg1_bits);
      put_bits(row, o, P.dg15_bits);
      put_bits(row, o, P.sa_bits);
      for (const auto& l : P.sig_limbs) { std::memcpy(row + 32 * o, l.data(), 8); o++; }
      for (const auto& l : P.pk_limbs) { std::memcpy(row + 32 * o, l.data(), 8); o++; }
      if (id) std::memcpy(row + 32 * o, id + 64, 80 * 32);  // slaveMerkleInclusionBranches
      o += 80;
      if (id) std::memcpy(row + 32 * o, id + 32, 32);  // skIdentity
      status[i] = PZK_PP_OK;
    } catch (const Fail& e) {
      std::memset(row, 0, row_bytes);
      status[i] = e.code;
    } catch (const std::exception&) {
      std::memset(row, 0, row_bytes);
      status[i] = PZK_PP_PARSE;
    }
  };
  int nt = threads;
  if (nt <= 0) {  // the CPUs this process may run on (a container's share, not the machine's count)
    cpu_set_t cs;
    nt = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : (int)std::thread::hardware_concurrency();
    nt = std::max(nt, 1);
  }
  nt = (int)std::min<size_t>((size_t)nt, std::max<size_t>(n, 1));
  if (nt <= 1) {
    for (size_t i = 0; i < n; i++) work(i);
    return 0;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; t++)
    pool.emplace_back([&, t]() { for (size_t i = t; i < n; i += (size_t)nt) work(i); });
  for (auto& th : pool) th.join();
  return 0;
}
