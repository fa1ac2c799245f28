// QueryIdentity(80) input offsets and template sizes, shared by the host layout builder (builder_query.cpp) and
// the device code (query.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pzk {

// main input offsets, in declaration order (queryIdentity.circom:51-77); after dg1 they depend on its length
// (744 bits for TD3, 760 for TD1: queryIdentityTD1.circom:75), see q_in_sib / q_in_ts / q_in_ic
enum QIn : int {
  QI_EVID = 0, QI_EVDATA, QI_ROOT, QI_SEL, QI_CUR, QI_TSLO, QI_TSHI, QI_ICLO, QI_ICHI, QI_BDLO, QI_BDHI, QI_EDLO, QI_EDHI,
  QI_CMASK, QI_SK, QI_PKPASS, QI_DG1, QI_SIB = QI_DG1 + 744, QI_TS = QI_SIB + 80, QI_IC, QI_N
};
constexpr int Q_DEPTH = 80;
// TD1 (queryIdentityTD1.circom with DG1TD1DataExtractor, dg1TD1DataExtractor.circom:5-107): 9 fields birthDate,
// expirationDate, name, nationality, citizenship, sex, documentNumber, personalNumber, documentType
constexpr int Q1_DG1 = 760, Q1_N = QI_N + 16;
constexpr int Q1_DGX_L[9] = {48, 48, 240, 24, 24, 8, 72, 88, 16};
constexpr int Q1_DGX_SHIFT[9] = {280, 344, 520, 400, 56, 336, 80, 160, 40};
// main output k + 1 (k < 9): extractor field Q1_OUT_FIELD[k] (or its PoseidonHash(1) for documentNumber /
// personalNumber) * selector bit Q1_OUT_SEL[k] (queryIdentityTD1.circom:97-105)
constexpr int Q1_OUT_SEL[9] = {1, 2, 3, 4, 5, 6, 7, 16, 17};
__host__ __device__ constexpr int q_dg1_len(bool td1) { return td1 ? Q1_DG1 : 744; }
__host__ __device__ constexpr int q_in_sib(bool td1) { return QI_DG1 + q_dg1_len(td1); }
__host__ __device__ constexpr int q_in_ts(bool td1) { return q_in_sib(td1) + Q_DEPTH; }
__host__ __device__ constexpr int q_in_ic(bool td1) { return q_in_ts(td1) + 1; }
__host__ __device__ constexpr int q_n_inputs(bool td1) { return q_in_ic(td1) + 1; }
// DG1DataExtractor field holding the citizenship / the dates; dg1 commitment chunk size
__host__ __device__ constexpr int q_f_cit(bool td1) { return td1 ? 4 : 5; }
__host__ __device__ constexpr int q_chunk(bool td1) { return td1 ? 190 : 186; }
// DG1DataExtractor fields (dg1DataExtractor.circom:20-96): birthDate, expirationDate, name, nameResidual,
// nationality, citizenship, sex, documentNumber = Bits2Num(L) with in[L-1-i] = dg1[SHIFT + i]
constexpr int Q_DGX_L[8] = {48, 48, 248, 64, 24, 24, 8, 72};
constexpr int Q_DGX_SHIFT[8] = {496, 560, 80, 328, 472, 56, 552, 392};
// main output k + 1 = extractor field k * selector bit Q_OUT_SEL[k] (queryIdentity.circom:86-93)
constexpr int Q_OUT_SEL[8] = {1, 2, 3, 3, 4, 5, 6, 7};
// template sizes (own signals + subcomponents)
constexpr uint32_t Q_SZ_DATEDEC = 17, Q_SZ_DIL = 109, Q_SZ_EDIL = 3 + 2 * Q_SZ_DATEDEC + Q_SZ_DIL,
                   Q_SZ_EDILN = 5 + 2 * Q_SZ_DATEDEC + 2 * Q_SZ_EDIL + Q_SZ_DIL, Q_SZ_FEIE = 9, Q_SZ_LT64 = 3 + 131,
                   Q_SZ_GEQ64 = 3 + Q_SZ_LT64, Q_SZ_CIT = 2 + 241 + 240, Q_SZ_CITEQ = 240 * 12;

}  // namespace pzk
