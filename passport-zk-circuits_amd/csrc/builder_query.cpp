// QueryIdentity(80) layout (identityManagement/queryIdentity.circom:37-229).
//
// main = QueryIdentity(80) {public [eventID .. citizenshipMask]}: the reference declares no main; its 14 public
// inputs are the ones declared before the private ones (queryIdentity.circom:51-69), so the witness order is
// the declaration order. Walks the component tree in creation order like builder_register.cpp; the CPU oracle
// (oracle/query.inc.c) derives every size independently and the parity tests compare every element.
// IdentityStateVerifier's BabyPbk is the reference's BabyjubjubBase8Multiplication.
#include "builder_impl.hpp"
#include "query_layout.hpp"

namespace pzk {

namespace {
uint32_t q_num2bits(int L) { return 2 * L + 1 + (L == 254 ? 254 + 383 + 271 : 0); }  // + AliasCheck
constexpr uint32_t SZ_ISEQUAL = 6, SZ_SWITCHER = 6;
}  // namespace

bool build_query(const pzk_params& p, Layout& L, std::string& why) {
  if (p.size_arg != 0 && p.size_arg != Q_DEPTH) {
    why = "QueryIdentity: idTreeDepth must be 80 (idStateSiblings[80] is fixed, queryIdentity.circom:75)";
    return false;
  }
  if (p.document_type != 0 && p.document_type != 1 && p.document_type != 3) {
    why = "QueryIdentity: document_type must be 3 (TD3, queryIdentity.circom) or 1 (TD1, queryIdentityTD1.circom)";
    return false;
  }
  const bool td1 = p.document_type == 1;
  const int NF = td1 ? 9 : 8, DG1L = q_dg1_len(td1), IN_SIB = q_in_sib(td1), IN_TS = q_in_ts(td1), IN_IC = q_in_ic(td1),
            CH = q_chunk(td1);
  auto fl = [&](int k) { return td1 ? Q1_DGX_L[k] : Q_DGX_L[k]; };
  auto fs = [&](int k) { return td1 ? Q1_DGX_SHIFT[k] : Q_DGX_SHIFT[k]; };
  Builder b(L);
  L.n_inputs = q_n_inputs(td1);
  L.n_outputs = td1 ? 10 : 9;
  L.n_public = 14;
  L.inputs = {{"eventID", QI_EVID, 1},
              {"eventData", QI_EVDATA, 1},
              {"idStateRoot", QI_ROOT, 1},
              {"selector", QI_SEL, 1},
              {"currentDate", QI_CUR, 1},
              {"timestampLowerbound", QI_TSLO, 1},
              {"timestampUpperbound", QI_TSHI, 1},
              {"identityCounterLowerbound", QI_ICLO, 1},
              {"identityCounterUpperbound", QI_ICHI, 1},
              {"birthDateLowerbound", QI_BDLO, 1},
              {"birthDateUpperbound", QI_BDHI, 1},
              {"expirationDateLowerbound", QI_EDLO, 1},
              {"expirationDateUpperbound", QI_EDHI, 1},
              {"citizenshipMask", QI_CMASK, 1},
              {"skIdentity", QI_SK, 1},
              {"pkPassportHash", QI_PKPASS, 1},
              {"dg1", QI_DG1, (uint64_t)DG1L},
              {"idStateSiblings", (uint64_t)IN_SIB, (uint64_t)Q_DEPTH},
              {"timestamp", (uint64_t)IN_TS, 1},
              {"identityCounter", (uint64_t)IN_IC, 1}};
  L.is_query = true;
  L.params = p;
  L.reg.in_br = IN_SIB;
  L.reg.in_root = QI_ROOT;
  L.reg.smt_check = 1;
  L.reg.q_td1 = td1 ? 1 : 0;
  L.bjj_core_fr = BJJ_CORE_FR;
  L.smt_core_fr = SMT_CORE_FR;

  // ---- value-store slots (Montgomery): loaded inputs, k_qry_prep outputs, chain outputs
  const int V_ONE = b.value(), V_SK = b.value(), V_EVID = b.value(), V_PKPASS = b.value(), V_IC = b.value(),
            V_TS = b.value(), V_SEL = b.value(), V_CMASK = b.value();
  int V_DGF[9], V_DGC[4], V_L[Q_DEPTH], V_R[Q_DEPTH];
  for (int k = 0; k < 9; k++) V_DGF[k] = b.value();
  for (int i = 0; i < 4; i++) V_DGC[i] = b.value();
  const int V_BJJ_X = b.value(), V_BJJ_Y = b.value();
  for (int i = 0; i < Q_DEPTH; i++) { V_L[i] = b.value(); V_R[i] = b.value(); }
  const int V_CIDX = b.value();
  const int V_CINV = b.value();
  for (int i = 1; i < 240; i++) b.value();
  for (auto [slot, in] : {std::pair<int, int>{V_SK, QI_SK}, {V_EVID, QI_EVID}, {V_PKPASS, QI_PKPASS}, {V_IC, IN_IC},
                          {V_TS, IN_TS}, {V_SEL, QI_SEL}, {V_CMASK, QI_CMASK}})
    L.loads.push_back(ValueLoad{slot, in});
  L.reg.v_one = V_ONE; L.reg.v_sk = V_SK; L.reg.v_dg1 = V_DGC[0]; L.reg.v_bjj = V_BJJ_X; L.reg.v_smt_lr = V_L[0];
  L.reg.q_dgf = V_DGF[0]; L.reg.q_cinv = V_CINV; L.reg.q_cidx = V_CIDX;
  // Poseidon levels: 0 sk hashes (and TD1's document / personal number hashes); 1 nullifier, dg1 commitment;
  // 2 (after the BabyJubJub core) pk identity hash, identity-state value; 3 tree position (the SMT key);
  // 4 SMTHash1 of the new leaf; 5 SMT level hashes

  // =========================== main: [1 | outputs | inputs | eventDataSquare] ===========================
  b.region(RK_ONE, 1);
  b.region(RK_Q_OUT, L.n_outputs);
  b.region(RK_INCOPY, L.n_inputs, {0});
  b.region(RK_Q_SQ, 1);
  // selectorBits = Num2Bits(18)(selector)
  b.region(RK_NUM2BITS, q_num2bits(18), {18, 0, V_SEL});
  // DG1DataExtractor / DG1TD1DataExtractor: fields | dg1 | Bits2Num encoders (in[L-1-i] = dg1[SHIFT + i])
  if (td1)
    b.region(RK_VALUE, 9, {-3, V_DGF[0], V_DGF[1], V_DGF[2], V_DGF[3], V_DGF[4], V_DGF[5], V_DGF[6], V_DGF[7], V_DGF[8]});
  else
    b.region(RK_VALUE, 8, {-3, V_DGF[0], V_DGF[1], V_DGF[2], V_DGF[3], V_DGF[4], V_DGF[5], V_DGF[6], V_DGF[7]});
  b.region(RK_INCOPY, DG1L, {QI_DG1});
  for (int k = 0; k < NF; k++) b.region(RK_BITS2NUM, q_num2bits(fl(k)), {fl(k), 0, QI_DG1 + fs(k) + fl(k) - 1, -1});
  if (td1) {  // documentNumberHasher, personalNumberHasher (queryIdentityTD1.circom:89-95)
    L.reg.q_doch = b.poseidon(1, {V_DGF[6]}, 0);
    L.reg.q_persh = b.poseidon(1, {V_DGF[7]}, 0);
  }
  // nullifier = Poseidon3(sk, Poseidon1(sk), eventID) (queryIdentity.circom:97-105)
  const int S_SKH = b.poseidon(1, {V_SK}, 0);
  const int S_NUL = b.poseidon(3, {V_SK, S_SKH, V_EVID}, 1);
  // timestamp / identity counter bounds (:107-149): GreaterEqThan(64) / LessThan(64) + ForceEqualIfEnabled
  for (int k = 0; k < 4; k++) {
    b.region(RK_Q_CMP, (k & 1) ? Q_SZ_LT64 : Q_SZ_GEQ64, {k});
    b.region(RK_Q_FEIE, Q_SZ_FEIE, {k});
  }
  // expiration date bounds (:151-169), birth date bounds (:171-189)
  for (int k = 0; k < 2; k++) {
    b.region(RK_Q_EDIL, Q_SZ_EDIL, {k});
    b.region(RK_Q_FEIE, Q_SZ_FEIE, {4 + k});
  }
  for (int k = 0; k < 2; k++) {
    b.region(RK_Q_EDILN, Q_SZ_EDILN, {k});
    b.region(RK_Q_FEIE, Q_SZ_FEIE, {6 + k});
  }
  // dg1Hasher (created before dg1Chunking[i]) = Poseidon5(4 x Bits2Num(186 | 190), skIndentityHasher) (:191-202)
  const size_t dgh_task = L.pos.size();
  const int S_DGC = b.poseidon(5, {V_DGC[0], V_DGC[1], V_DGC[2], V_DGC[3], -1}, 1);
  for (int i = 0; i < 4; i++) b.region(RK_BITS2NUM, q_num2bits(CH), {CH, 0, QI_DG1 + CH * i, 1});
  const int S_SKH2 = b.poseidon(1, {V_SK}, 0);
  L.pos[dgh_task].in_slot[4] = S_SKH2;

  // =========================== IdentityStateVerifier(80) (identityStateVerifier.circom:8-46) ===========================
  // own: skIdentity, pkPassHash, dgCommit, identityCounter, timestamp, idStateRoot, idStateSiblings[80] | treePosition
  b.region(RK_INCOPY, 2, {QI_SK});  // skIdentity, pkPassportHash (adjacent inputs)
  b.region(RK_VALUE, 1, {S_DGC});
  b.region(RK_INCOPY, 1, {IN_IC});
  b.region(RK_INCOPY, 1, {IN_TS});
  b.region(RK_INCOPY, 1, {QI_ROOT});
  b.region(RK_INCOPY, Q_DEPTH, {IN_SIB});
  const uint32_t r_pos = b.region(RK_VALUE, 1, {-1, -1});  // treePosition (slot patched below)
  // babyPbk: BabyjubjubBase8Multiplication: out[2] | scalar | getBase8, num2Bits(254), adders/doublers
  b.region(RK_BJJ_OWN, 3 + 2);
  b.region(RK_NUM2BITS, q_num2bits(254), {254, 0, V_SK});
  b.region(RK_BJJ_STEPS, 46 + 253 * 60);
  const int S_PKID = b.poseidon(2, {V_BJJ_X, V_BJJ_Y}, 2);
  const int S_POS = b.poseidon(2, {V_PKPASS, S_PKID}, 3);
  const int S_VAL = b.poseidon(3, {S_DGC, V_IC, V_TS}, 2);
  // SMTVerifier(80): isVerified | root, leaf, key, siblings[80] | value | hash1New, n2bNew, smtLevIns, sm[80],
  // levels[79..0], isEqual
  b.region(RK_SMT_OWN, 1 + 3 + Q_DEPTH + 1, {QI_ROOT, IN_SIB});
  b.region(RK_SMTHASH, 3, {-1});
  const int S_LEAF = b.poseidon(3, {S_POS, S_VAL, V_ONE}, 4);
  b.region(RK_NUM2BITS, q_num2bits(254), {254, 0, S_POS});
  b.region(RK_LEVINS, Q_DEPTH + Q_DEPTH + (Q_DEPTH - 1) + Q_DEPTH * 3, {IN_SIB});
  b.region(RK_SM, Q_DEPTH * 4);
  int S_H[Q_DEPTH];
  for (int i = 0; i < Q_DEPTH; i++) S_H[i] = b.value();
  for (int i = Q_DEPTH - 1; i >= 0; i--) {
    b.region(RK_SMT_LEVEL, 8, {i, IN_SIB});
    b.region(RK_SMTHASH, 3, {i});
    b.poseidon(2, {V_L[i], V_R[i]}, 5, S_H[i]);
    L.pos.back().smt_level = i;
    b.region(RK_SWITCHER, SZ_SWITCHER, {i, IN_SIB});
  }
  b.region(RK_ISEQ_ROOT, SZ_ISEQUAL, {QI_ROOT});
  for (int i = 1; i < Q_DEPTH; i++)
    if (S_H[i] != S_H[0] + i) { why = "internal: SMT hash slots not contiguous"; return false; }

  // =========================== CitizenshipCheck (citizenshipCheck.circom:6-275) ===========================
  b.region(RK_Q_CIT, Q_SZ_CIT);
  b.region(RK_NUM2BITS, q_num2bits(240), {240, 0, V_CMASK});
  b.region(RK_Q_CITEQ, Q_SZ_CITEQ);

  L.reg.q_nul = S_NUL;
  L.reg.v_pkhash = S_POS;
  L.reg.v_leaf = S_LEAF;
  L.reg.v_smt_h = S_H[0];
  L.reg.v_smt_key = S_POS;
  L.reg.v_smt_val = S_VAL;
  L.regions[r_pos].a[1] = S_POS;
  L.out_slots = {S_NUL};
  b.finalize();
  return true;
}

}  // namespace pzk
