// Launch templates of the alternative GEMM configurations (gemm_core.h kernel), shared by the
// translation units that instantiate them (gemm_w4.hip, gemm_alt_bp.hip, gemm_alt_t.hip: one
// TU per configuration family so the heavy instantiations compile in parallel).
#pragma once
#include "gemm_core.h"

namespace pra {
namespace {

template <typename CF, typename T, bool AK, bool BK, int E>
void launch_w4(const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum, int M, int N, int K,
               int lda, int ldb, int ldc, int ldz, int beta, int splits, float* ws, hipStream_t s) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  auto pa = static_cast<const uint16_t*>(A);
  auto pb = static_cast<const uint16_t*>(B);
  if (splits > 1) {
    gemm_lds_kernel<T, CF, AK, BK, kNone, false, true><<<tiles * splits, CF::NT, 0, s>>>(
        pa, pb, nullptr, nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, ldz, splits, ws);
    return;  // the caller runs the split-K combine
  }
  auto pbias = static_cast<const uint16_t*>(bias);
  auto pc = static_cast<uint16_t*>(C);
  auto pz = static_cast<uint16_t*>(Z);
  if (beta)
    gemm_lds_kernel<T, CF, AK, BK, E, true, false><<<tiles, CF::NT, 0, s>>>(pa, pb, pbias, pc, pz, colsum, M, N, K,
                                                                            lda, ldb, ldc, ldz, 1, nullptr);
  else
    gemm_lds_kernel<T, CF, AK, BK, E, false, false><<<tiles, CF::NT, 0, s>>>(pa, pb, pbias, pc, pz, colsum, M, N, K,
                                                                             lda, ldb, ldc, ldz, 1, nullptr);
}

template <typename CF, typename T, bool AK, bool BK>
int launch_w4_l(const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum, int M, int N, int K,
                int lda, int ldb, int ldc, int ldz, int epi, int beta, int splits, float* ws, hipStream_t s) {
  switch (epi) {
    case kNone: launch_w4<CF, T, AK, BK, kNone>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); return 0;
    case kGeluErf: launch_w4<CF, T, AK, BK, kGeluErf>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); return 0;
    case kGeluTanh: launch_w4<CF, T, AK, BK, kGeluTanh>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); return 0;
    case kDGeluErf: launch_w4<CF, T, AK, BK, kDGeluErf>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); return 0;
    case kDGeluTanh: launch_w4<CF, T, AK, BK, kDGeluTanh>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); return 0;
    case kGeluErfD:
      if constexpr (AK && !BK) { launch_w4<CF, T, AK, BK, kGeluErfD>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); return 0; }
      return -1;
    case kGeluTanhD:
      if constexpr (AK && !BK) { launch_w4<CF, T, AK, BK, kGeluTanhD>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); return 0; }
      return -1;
    case kMulZ:
      if constexpr (AK && BK) { launch_w4<CF, T, AK, BK, kMulZ>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); return 0; }
      return -1;
    default: return -1;  // (ReLU: the 8-wave kernel)
  }
}

template <typename CF>
int launch_alt(int layout, const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum, int M,
               int N, int K, int lda, int ldb, int ldc, int ldz, int dtype, int epi, int beta, int splits, float* ws,
               hipStream_t s) {
  if (dtype != kBF16) return -1;
  switch (layout) {
    case 0: return launch_w4_l<CF, bf16, true, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, splits, ws, s);
    case 1: return launch_w4_l<CF, bf16, true, true>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, splits, ws, s);
    case 2: return launch_w4_l<CF, bf16, false, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, splits, ws, s);
    default: return -1;
  }
}

}  // namespace
}  // namespace pra

// One configuration's entry (same contract as pra_gemm_lds; bf16 only; splits > 1 launches only
// the partial-tile pass into ws).
#define PRA_GEMM_ALT_ENTRY(NAME, CFG)                                                                      \
  extern "C" int NAME(int layout, const void* A, const void* B, const void* bias, void* C, void* Z,           \
                      float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype,      \
                      int epi, int beta, int splits, float* ws, hipStream_t s) {                              \
    return pra::launch_alt<CFG>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi,  \
                                beta, splits, ws, s);                                                         \
  }
