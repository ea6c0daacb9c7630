// 4-wave configuration of the LDS-DMA MFMA GEMM (gemm_core.h): 256x256 output tile per
// 256-thread workgroup, 2 x 2 waves of 128x128 outputs each, i.e. ONE wave per SIMD holding 64
// 16x16 fp32 accumulator tiles (all 256 AGPRs) with double-buffered 128-row A and B fragments
// in VGPRs. Against the 8-wave 128x64-per-wave layout this halves the LDS fragment bytes read
// per MFMA (8 A + 8 B ds_read_b128 per 64 MFMAs instead of 8 + 4 per 32) — the configuration
// hipBLASLt's fastest gfx950 dy·Wᵀ kernel uses (MT256x256x64, MI16x16, 4 waves). Epilogues,
// split-K and the LDS-staged output stream are the shared template's.
// The same file instantiates W8I: the 8-wave layout with the W4 one-filler-per-MFMA segment
// schedule (A/B against the burst schedule of gemm_lds.hip's W8).
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
    default: return -1;  // (ReLU: the 8-wave kernel)
  }
}

using W8I = WCfg<2, 4, 256, 256, true>;
using W4B = WCfg<2, 2, 256, 256, true, true>;   // W4 with MUBUF operand DMA
using W8B = WCfg<2, 4, 256, 256, false, true>;  // W8 (burst schedule) with MUBUF operand DMA
using W4P = WCfg<2, 2, 256, 256, true, false, true>;  // W4 with the two-barrier early-refill schedule
using W8P = WCfg<2, 4, 256, 256, true, false, true>;  // W8 with the two-barrier early-refill schedule
using W4T = WCfg<2, 2, 256, 256, true, false, false, true>;  // W4 with the TS schedule (kstep_t)
using W8T = WCfg<2, 4, 256, 256, true, false, false, true>;  // W8 with the TS schedule

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

// Same contract as pra_gemm_lds (validated there); bf16 only. splits > 1 launches only the
// partial-tile pass into ws (the caller combines). Returns -1 for what it does not cover.
extern "C" int pra_gemm_w4(int layout, const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum,
                           int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype, int epi, int beta,
                           int splits, float* ws, hipStream_t s) {
  return pra::launch_alt<pra::W4>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta,
                                  splits, ws, s);
}

extern "C" int pra_gemm_w8i(int layout, const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum,
                            int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype, int epi, int beta,
                            int splits, float* ws, hipStream_t s) {
  return pra::launch_alt<pra::W8I>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta,
                                   splits, ws, s);
}

// cfg: 0 = W4, 1 = W8I, 2 = W4B, 3 = W8B, 4 = W4P, 5 = W8P, 6 = W4T, 7 = W8T
extern "C" int pra_gemm_alt(int cfg, int layout, const void* A, const void* B, const void* bias, void* C, void* Z,
                            float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype, int epi,
                            int beta, int splits, float* ws, hipStream_t s) {
  switch (cfg) {
    case 0: return pra::launch_alt<pra::W4>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
    case 1: return pra::launch_alt<pra::W8I>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
    case 2: return pra::launch_alt<pra::W4B>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
    case 3: return pra::launch_alt<pra::W8B>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
    case 4: return pra::launch_alt<pra::W4P>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
    case 5: return pra::launch_alt<pra::W8P>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
    case 6: return pra::launch_alt<pra::W4T>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
    case 7: return pra::launch_alt<pra::W8T>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
    default: return -1;
  }
}
