// QueryIdentity(80) input offsets and template sizes, shared by the host layout builder (builder_query.cpp) and
// the device code (query.hpp).
#pragma once
#include <stdint.h>

namespace pzk {

// main input offsets, in declaration order (queryIdentity.circom:51-77)
enum QIn : int {
  QI_EVID = 0, QI_EVDATA, QI_ROOT, QI_SEL, QI_CUR, QI_TSLO, QI_TSHI, QI_ICLO, QI_ICHI, QI_BDLO, QI_BDHI, QI_EDLO, QI_EDHI,
  QI_CMASK, QI_SK, QI_PKPASS, QI_DG1, QI_SIB = QI_DG1 + 744, QI_TS = QI_SIB + 80, QI_IC, QI_N
};
constexpr int Q_DEPTH = 80;
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
