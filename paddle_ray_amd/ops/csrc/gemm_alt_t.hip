// TS-schedule GEMM configurations (gemm_core.h kstep_t; dispatcher in gemm_w4.hip).
#include "gemm_alt.h"

namespace pra {
namespace {
using W4T = WCfg<2, 2, 256, 256, true, false, false, true>;  // W4 with the TS schedule
using W8T = WCfg<2, 4, 256, 256, true, false, false, true>;  // W8 with the TS schedule
}  // namespace
}  // namespace pra

PRA_GEMM_ALT_ENTRY(pra_gemm_w4t, pra::W4T)
PRA_GEMM_ALT_ENTRY(pra_gemm_w8t, pra::W8T)

// Two weight gradients C1 (+)= A1ᵀ·B1 [M x N1] and C2 (+)= A2ᵀ·B2 [M x N2] (layout 2, shared M and
// K) in ONE launch of the W8T kernel (gemm_core.h GemmG2), no split-K. Returns -1 (nothing
// launched) for shapes outside the kernel's assumptions.
extern "C" int pra_gemm_tn_grouped2(const void* A1, const void* B1, void* C1, int N1, int lda1, int ldb1, int ldc1,
                                    const void* A2, const void* B2, void* C2, int N2, int lda2, int ldb2, int ldc2,
                                    int M, int K, int beta, hipStream_t s) {
  if (M < 8 || (M & 7) || (K & 63) || K <= 0 || (N1 & 7) || (N2 & 7) || N1 < 8 || N2 < 8) return -1;
  if ((lda1 | ldb1 | ldc1 | lda2 | ldb2 | ldc2) & 7) return -1;
  const int tm = (M + pra::BM - 1) / pra::BM;
  const int t1 = tm * ((N1 + pra::BN - 1) / pra::BN), t2 = tm * ((N2 + pra::BN - 1) / pra::BN);
  pra::GemmG2 g{static_cast<const uint16_t*>(A2), static_cast<const uint16_t*>(B2), static_cast<uint16_t*>(C2),
                N2, lda2, ldb2, ldc2, t1};
  auto a = static_cast<const uint16_t*>(A1);
  auto b = static_cast<const uint16_t*>(B1);
  auto c = static_cast<uint16_t*>(C1);
  if (beta)
    pra::gemm_lds_kernel<pra::bf16, pra::W8T, false, false, pra::kNone, true, false><<<t1 + t2, pra::W8T::NT, 0, s>>>(
        a, b, nullptr, c, nullptr, nullptr, M, N1, K, lda1, ldb1, ldc1, N1, 1, nullptr, {}, nullptr, nullptr, nullptr, g);
  else
    pra::gemm_lds_kernel<pra::bf16, pra::W8T, false, false, pra::kNone, false, false><<<t1 + t2, pra::W8T::NT, 0, s>>>(
        a, b, nullptr, c, nullptr, nullptr, M, N1, K, lda1, ldb1, ldc1, N1, 1, nullptr, {}, nullptr, nullptr, nullptr, g);
  return 0;
}
