// Layout builder (see builder.hpp). Template sizes follow the circom sources cited inline;
// every offset here is re-derived independently of the CPU oracle, and the parity tests
// compare the two layouts element by element.
#include "builder_impl.hpp"
#include "sha_prog.hpp"
#include "pos_prog.hpp"

#include <algorithm>
#include <map>

namespace pzk {

// Descriptors of the 150,762 signals of one SHA-256 block, in witness order (sha_prog.hpp).
// Mirrors the template signal order of sha256Schedule.circom:11-72, sha256Rounds.circom:12-125
// and sha256Compress.circom:11-96; the GPU tests check every emitted element against the oracle.
void sha_program(std::vector<uint32_t>& P) {
  P.clear();
  P.reserve(SHA_BLOCK_SIGNALS_COUNT);
  auto X = [&](int idx, int lo, int n) { P.push_back(sha_desc(idx, lo, n, SHA_D_EXTRACT)); };
  auto M = [&](int idx, int lo, int n) { P.push_back(sha_desc(idx, lo, n, SHA_D_MASK)); };
  auto bits32 = [&](int idx) { for (int i = 0; i < 32; i++) X(idx, i, 1); };
  // GetSumOfNElements(32) of (1<<i)*bit_i(X): out | in[32] | sum[31]
  auto getsum32 = [&](int idx) {
    X(idx, 0, 64);
    for (int j = 1; j <= 32; j++) M(idx, j - 1, 1);
    for (int j = 33; j < 64; j++) M(idx, 0, j - 31);
  };
  // GetLastNBits(32) of V: div | out[32] | in | check[32] | GetLastBitUnsecure[32] (in, out, div)
  auto lastnbits32 = [&](int idx) {
    X(idx, 32, 64);
    for (int j = 1; j <= 32; j++) X(idx, j - 1, 1);
    X(idx, 0, 64);
    for (int j = 34; j < 66; j++) M(idx, 0, j - 33);
    for (int q = 0; q < 32; q++) { X(idx, q, 1); X(idx, q + 1, 64); X(idx, q, 64); }
  };
  // Bits2Num(32): out | in[32] | sum[32]
  auto bits2num32 = [&](int idx) {
    X(idx, 0, 64);
    for (int j = 1; j <= 32; j++) X(idx, j - 1, 1);
    for (int j = 33; j <= 64; j++) M(idx, 0, j - 32);
  };
  auto hin = [](int j) { return j < 4 ? sha_wt_a(-j) : sha_wt_e(4 - j); };
  // ---- Sha2_224_256Shedule
  for (int k = 0; k < 64; k++) X(SHA_WT_W + k, 0, 64);                 // outWords
  for (int k = 0; k < 16; k++) bits32(SHA_WT_W + k);                   // chunkBits[16][32]
  for (int k = 0; k < 64; k++) bits32(SHA_WT_W + k);                   // outBits[64][32]
  for (int k = 0; k < 16; k++) getsum32(SHA_WT_W + k);                 // sumN[16]
  for (int r = 0; r < 48; r++) {
    const int b = SHA_WT_SCH + SHA_SCH_WORDS * r;
    getsum32(b + SW_S0);
    getsum32(b + SW_S1);
    for (int i = 0; i < 32; i++) {  // s0Xor[i], s1Xor[i]: XOR3_v2 out | x, y, z | tmp
      X(b + SW_S0, i, 1); X(b + SW_X7, i, 1); X(b + SW_Y18, i, 1); X(b + SW_Z3, i, 1); X(b + SW_T0, i, 1);
      X(b + SW_S1, i, 1); X(b + SW_X17, i, 1); X(b + SW_Y19, i, 1); X(b + SW_Z10, i, 1); X(b + SW_T1, i, 1);
    }
    lastnbits32(b + SW_V);
    bits2num32(SHA_WT_W + r + 16);
  }
  // ---- Sha2_224_256Rounds(64): own signals
  for (int j = 0; j < 8; j++)
    for (int i = 0; i < 32; i++) X(SHA_WT_FF32 + j, i, 1);          // outHash[8][32]
  for (int k = 0; k < 64; k++) X(SHA_WT_W + k, 0, 64);                 // words
  for (int j = 0; j < 8; j++) bits32(hin(j));                          // hashBits
  for (int arr = 0; arr < 3; arr++)                                    // a, b, c [65][32]
    for (int k = 0; k < 65; k++) bits32(sha_wt_a(k - arr));
  for (int k = 0; k < 65; k++) X(sha_wt_a(k - 3), 0, 64);              // dd
  for (int arr = 0; arr < 3; arr++)                                    // e, f, g [65][32]
    for (int k = 0; k < 65; k++) bits32(sha_wt_e(k - arr));
  for (int k = 0; k < 65; k++) X(sha_wt_e(k - 3), 0, 64);              // hh
  for (int k = 0; k < 64; k++) X(SHA_WT_K + k, 0, 64);                 // ROUND_KEYS
  for (int j = 0; j < 8; j++) X(hin(j), 0, 64);                        // hashWords
  // subcomponents: round keys, sumDd, sumHh, sum[8], compress[64], modulo[8], sumA..sumG
  for (int k = 0; k < 64; k++) X(SHA_WT_K + k, 0, 64);
  getsum32(hin(3));
  getsum32(hin(7));
  for (int j = 0; j < 8; j++) getsum32(hin(j));
  for (int k = 0; k < 64; k++) {
    const int a = sha_wt_a(k), bb = sha_wt_a(k - 1), c = sha_wt_a(k - 2), d = sha_wt_a(k - 3);
    const int e = sha_wt_e(k), f = sha_wt_e(k - 1), g = sha_wt_e(k - 2), h = sha_wt_e(k - 3);
    const int cw = SHA_WT_CMP + SHA_CMP_WORDS * k;
    // outputs: outA bits, a bits, b bits, c | outE bits, e bits, f bits, g
    bits32(sha_wt_a(k + 1)); bits32(a); bits32(bb); X(c, 0, 64);
    bits32(sha_wt_e(k + 1)); bits32(e); bits32(f); X(g, 0, 64);
    // inputs: inp, key, a, b, c bits, d | e, f, g bits, h
    X(SHA_WT_W + k, 0, 64); X(SHA_WT_K + k, 0, 64);
    bits32(a); bits32(bb); bits32(c); X(d, 0, 64);
    bits32(e); bits32(f); bits32(g); X(h, 0, 64);
    bits32(cw + CW_CH);                                                // ch bits
    X(cw + CW_OVE, 0, 64); X(cw + CW_OVA, 0, 64);
    getsum32(c); getsum32(g); getsum32(cw + CW_S0); getsum32(cw + CW_S1); getsum32(cw + CW_MJ);
    getsum32(cw + CW_CH);
    for (int i = 0; i < 32; i++) {  // Bits2(a+b+c) | XOR3 Sigma0 | XOR3 Sigma1
      X(cw + CW_XY, 2 * i, 1); X(cw + CW_XY, 2 * i + 1, 1); X(cw + CW_XY, 2 * i, 2);
      X(cw + CW_S0, i, 1); X(cw + CW_R2, i, 1); X(cw + CW_R13, i, 1); X(cw + CW_R22, i, 1); X(cw + CW_T0, i, 1);
      X(cw + CW_S1, i, 1); X(cw + CW_R6, i, 1); X(cw + CW_R11, i, 1); X(cw + CW_R25, i, 1); X(cw + CW_T1, i, 1);
    }
    lastnbits32(cw + CW_OVE);
    lastnbits32(cw + CW_OVA);
  }
  for (int j = 0; j < 8; j++) lastnbits32(SHA_WT_FF64 + j);            // modulo[8]
  for (int q = 0; q < 6; q++) getsum32(q < 3 ? sha_wt_a(64 - q) : sha_wt_e(64 - (q - 3)));  // sumA..sumG
}

// Descriptors of the signals of a PoseidonHash(t-1) block (pos_prog.hpp), in witness order:
// PoseidonHash own (out, in[n]), PoseidonEx own (out, in[n], initialState), ark[0], then per
// full round Sigma[t] (out, in, in2, in4), Ark (out[t], in[t]), Mix (out[t], in[t], t x GetSum),
// per partial round SigmaP and MixS, finally Sigma[7] and MixLast (poseidon.circom:80-209).
void pos_program(int t, std::vector<uint16_t>& P) {
  const PosImg I(t);
  const int n = t - 1, RP = I.rp;
  P.clear();
  auto C = [&](int idx) { P.push_back(pos_desc(idx)); };
  // GetSumOfNElements(t) over a prefix-sum row: out | in[t] (the products) | sum[t-1]
  auto getsum = [&](int row) {
    const int r = row < I.ps ? (row - I.fs) / t : 7 * t + 1 + (row - I.ps) / t;  // phase-B row number
    C(row + t - 1);
    C(row);
    for (int j = 1; j < t; j++) C(I.prod(r, j));
    for (int q = 1; q < t; q++) C(row + q);
  };
  C(I.hash);
  for (int i = 0; i < n; i++) C(I.inp + i);
  C(I.hash);
  for (int i = 0; i < n; i++) C(I.inp + i);
  C(I.zero);
  for (int j = 0; j < t; j++) C(I.in + j);                   // ark[0].out
  C(I.zero);                                                 // ark[0].in = initialState, inputs
  for (int i = 0; i < n; i++) C(I.inp + i);
  auto full_round = [&](int f) {
    for (int j = 0; j < t; j++) { int i = f * t + j; C(I.p5 + i); C(I.in + i); C(I.p2 + i); C(I.p4 + i); }
    for (int q = 0; q < t; q++) C(I.ark + f * t + q);        // ark[f+1].out
    for (int q = 0; q < t; q++) C(I.p5 + f * t + q);         // ark[f+1].in
    for (int q = 0; q < t; q++) C(f == 3 ? I.pin + q : I.in + (f + 1) * t + q);  // mix.out = next layer
    for (int q = 0; q < t; q++) C(I.ark + f * t + q);        // mix.in
    for (int i = 0; i < t; i++) getsum(I.fs + (f * t + i) * t);
  };
  for (int f = 0; f < 4; f++) full_round(f);
  for (int r = 0; r < RP; r++) {
    C(I.pp5 + r); C(I.pin + r * t); C(I.pp2 + r); C(I.pp4 + r);      // sigmaP
    for (int q = 0; q < t; q++) C(I.pin + (r + 1) * t + q);          // mixS.out
    C(I.pin0 + r);                                                   // mixS.in
    for (int i = 1; i < t; i++) C(I.pin + r * t + i);
    getsum(I.ps + r * t);
  }
  for (int f = 4; f < 7; f++) full_round(f);
  for (int j = 0; j < t; j++) { int i = 7 * t + j; C(I.p5 + i); C(I.in + i); C(I.p2 + i); C(I.p4 + i); }
  C(I.hash);                                                         // mixLast
  for (int j = 0; j < t; j++) C(I.p5 + 7 * t + j);
  getsum(I.ls);
}

namespace {

bool build_poseidon(const pzk_params& p, Layout& L, std::string& why) {
  int n = p.size_arg;
  if (n < 1 || n > 5) { why = "PoseidonHash(n): n must be 1..5 (Poseidon parameters shipped for t = 2..6)"; return false; }
  Builder b(L);
  L.n_inputs = n;
  L.n_outputs = 1;
  L.inputs.push_back({"in", 0, (uint64_t)n});
  std::vector<int> slots;
  for (int i = 0; i < n; i++) { int s = b.value(); slots.push_back(s); L.loads.push_back(ValueLoad{s, i}); }
  b.region(RK_ONE, 1);
  b.poseidon(n, slots, 0);  // main = PoseidonHash(n): [1, out, in[n], PoseidonEx]
  b.finalize();
  return true;
}

bool build_sha256(const pzk_params& p, Layout& L, std::string& why) {
  int B = p.size_arg;
  if (B < 1 || B > 64) { why = "Sha256HashChunks(blocks): blocks must be 1..64"; return false; }
  Builder b(L);
  L.n_inputs = 512ull * B;
  L.n_outputs = 256;
  L.inputs.push_back({"in", 0, L.n_inputs});
  b.region(RK_ONE, 1);
  b.sha256(0, B, false);
  b.finalize();
  return true;
}

bool build_sha1(const pzk_params& p, Layout& L, std::string& why) {
  int B = p.size_arg;
  if (B < 1 || B > 64) { why = "Sha1HashChunks(blocks): blocks must be 1..64"; return false; }
  Builder b(L);
  L.n_inputs = 512ull * B;
  L.n_outputs = 160;
  L.inputs.push_back({"in", 0, L.n_inputs});
  b.region(RK_ONE, 1);
  b.sha1(0, B);
  b.finalize();
  return true;
}

bool build_sha512(const pzk_params& p, Layout& L, std::string& why, int O) {
  int B = p.size_arg;
  if (B < 1 || B > 16) { why = "Sha384/Sha512HashChunks(blocks): blocks must be 1..16"; return false; }
  Builder b(L);
  L.n_inputs = 1024ull * B;
  L.n_outputs = O;
  L.inputs.push_back({"in", 0, L.n_inputs});
  b.region(RK_ONE, 1);
  b.sha512(0, B, O);
  b.finalize();
  return true;
}

}  // namespace

bool build_register(const pzk_params& p, Layout& L, std::string& why);

bool build_layout(const pzk_params& p, Layout& L, std::string& why) {
  L = Layout();
  bool ok;
  switch (p.circuit) {
    case PZK_CIRCUIT_POSEIDON: ok = build_poseidon(p, L, why); break;
    case PZK_CIRCUIT_SHA256: ok = build_sha256(p, L, why); break;
    case PZK_CIRCUIT_SHA1: ok = build_sha1(p, L, why); break;
    case PZK_CIRCUIT_SHA384: ok = build_sha512(p, L, why, 384); break;
    case PZK_CIRCUIT_SHA512: ok = build_sha512(p, L, why, 512); break;
    case PZK_CIRCUIT_REGISTER: ok = build_register(p, L, why); break;
    case PZK_CIRCUIT_QUERY: ok = build_query(p, L, why); break;
    default: why = "unknown circuit family"; return false;
  }
  if (ok && !L.pos.empty()) {
    L.pos_prog.clear();
    for (int t = 2; t <= POS_MAX_T; t++) {
      std::vector<uint16_t> P;
      pos_program(t, P);
      if (P.size() != pos_hash_size(t - 1)) { why = "internal: Poseidon block program size"; return false; }
      L.pos_prog_off[t] = (uint32_t)L.pos_prog.size();
      L.pos_prog.insert(L.pos_prog.end(), P.begin(), P.end());
    }
  }
  if (ok && !L.sha.empty()) {
    sha_program(L.sha_prog);
    if (L.sha_prog.size() != SHA_BLOCK_SIGNALS_COUNT) { why = "internal: SHA block program size"; return false; }
  }
  return ok;
}

}  // namespace pzk
