// 4-wave configuration of the LDS-DMA MFMA GEMM (gemm_core.h): 256x256 output tile per
// 256-thread workgroup, 2 x 2 waves of 128x128 outputs each, i.e. ONE wave per SIMD holding 64
// 16x16 fp32 accumulator tiles (all 256 AGPRs) with double-buffered 128-row A and B fragments
// in VGPRs. Against the 8-wave 128x64-per-wave layout this halves the LDS fragment bytes read
// per MFMA (8 A + 8 B ds_read_b128 per 64 MFMAs instead of 8 + 4 per 32) — the configuration
// hipBLASLt's fastest gfx950 dy·Wᵀ kernel uses (MT256x256x64, MI16x16, 4 waves). Epilogues,
// split-K and the LDS-staged output stream are the shared template's.
// The same file instantiates W8I: the 8-wave layout with the W4 one-filler-per-MFMA segment
// schedule (A/B against the burst schedule of gemm_lds.hip's W8), and holds the configuration
// dispatcher; the other families live in gemm_alt_bp.hip / gemm_alt_t.hip.
#include "gemm_alt.h"

namespace pra {
namespace {
using W8I = WCfg<2, 4, 256, 256, true>;
}  // namespace
}  // namespace pra

PRA_GEMM_ALT_ENTRY(pra_gemm_w4, pra::W4)
PRA_GEMM_ALT_ENTRY(pra_gemm_w8i, pra::W8I)

#define PRA_ALT_DECL(NAME)                                                                                  \
  extern "C" int NAME(int, const void*, const void*, const void*, void*, void*, float*, int, int, int, int,   \
                      int, int, int, int, int, int, int, float*, hipStream_t);
PRA_ALT_DECL(pra_gemm_w4b)
PRA_ALT_DECL(pra_gemm_w8b)
PRA_ALT_DECL(pra_gemm_w4p)
PRA_ALT_DECL(pra_gemm_w8p)
PRA_ALT_DECL(pra_gemm_w4t)
PRA_ALT_DECL(pra_gemm_w8t)

// cfg: 0 = W4, 1 = W8I, 2 = W4B, 3 = W8B, 4 = W4P, 5 = W8P, 6 = W4T, 7 = W8T
extern "C" int pra_gemm_alt(int cfg, int layout, const void* A, const void* B, const void* bias, void* C, void* Z,
                            float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype, int epi,
                            int beta, int splits, float* ws, hipStream_t s) {
  static decltype(&pra_gemm_w4) const fns[8] = {pra_gemm_w4,  pra_gemm_w8i, pra_gemm_w4b, pra_gemm_w8b,
                                                pra_gemm_w4p, pra_gemm_w8p, pra_gemm_w4t, pra_gemm_w8t};
  if (cfg < 0 || cfg >= 8) return -1;
  return fns[cfg](layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, dtype, epi, beta, splits, ws, s);
}
