// Launch side of the persistent TS GEMM (gemm_pts.h): one translation unit per wave configuration.
#pragma once
#include <mutex>
#include <utility>
#include <vector>

#include "gemm_pts.h"

namespace pra {
namespace {
using W4T = WCfg<2, 2, 256, 256, true, false, false, true>;
using W8T = WCfg<2, 4, 256, 256, true, false, false, true>;

int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// measurement variant of the plain (no epilogue) kernel: PRA_PTS_VAR (gemm_pts.h VAR; 0 = default)
int pts_var() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PRA_PTS_VAR");
    v = e ? atoi(e) : 0;
  }
  return v;
}

// Dynamic tile order (gemm_pts.h tctr), default on (PRA_PTS_DYN=0: the static order). Under a
// 32-workgroup co-resident load the fused fc1 GEMM took 1.60x its time with the static order and
// 1.17x with the dynamic one (profiles/r6/pts_dynamic_order.md). A block holds the 8 per-XCD
// counters; it starts zeroed and each XCD's last fetch re-zeroes its counter, so no memset is
// launched per GEMM and graph replays find it ready.
// PRA_PTS_NT: which epilogue stores carry the non-temporal hint (see launch_pts). Default 3: the
// fused-epilogue GEMMs' C and Z (fc1 forward + gelu' 562 -> 544 us, fc2 dgrad * gelu' 546 -> 535 us
// alone); plain GEMMs keep L2-allocating stores (their outputs are read next: nt on the dy·Wᵀ
// out-projection dgrad cost 101 -> 108 us). GPT step 125.8 -> 125.6 ms (profiles/r6/pts_nt_stores.md).
int pts_nt() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PRA_PTS_NT");
    v = e ? atoi(e) : 3;
  }
  return v;
}
int pts_dyn() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PRA_PTS_DYN");
    v = e ? atoi(e) : 1;
  }
  return v;
}
// Counter blocks come from one zeroed pool per device, allocated at the first launch outside a
// stream capture (hipMalloc would invalidate a capture). Eager launches use one block per stream
// (launches on a stream are ordered, so they can share it); every captured launch takes a block
// of its own, so graphs replayed concurrently never share counters. With no pool yet, or the
// pool used up, a captured launch falls back to the static order.
constexpr int kPtsSlotInts = 8 * kPtsCtrStride, kPtsSlots = 1024;
int* pts_counters(hipStream_t s) {
  struct Pool {
    int dev;
    int* base;
    int used;
    std::vector<std::pair<hipStream_t, int>> eager;
  };
  static std::mutex mu;
  static std::vector<Pool> pools;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess) return nullptr;
  const bool capturing = cs != hipStreamCaptureStatusNone;
  std::lock_guard<std::mutex> lk(mu);
  Pool* p = nullptr;
  for (auto& q : pools)
    if (q.dev == dev) p = &q;
  if (!p) {
    if (capturing) return nullptr;
    int* base = nullptr;
    const size_t bytes = size_t(kPtsSlots) * kPtsSlotInts * sizeof(int);
    if (hipMalloc(&base, bytes) != hipSuccess) return nullptr;
    if (hipMemset(base, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(base);
      return nullptr;
    }
    pools.push_back(Pool{dev, base, 0, {}});
    p = &pools.back();
  }
  if (!capturing)
    for (auto& e : p->eager)
      if (e.first == s) return p->base + size_t(e.second) * kPtsSlotInts;
  if (p->used >= kPtsSlots) return nullptr;
  const int slot = p->used++;
  if (!capturing) p->eager.emplace_back(s, slot);
  return p->base + size_t(slot) * kPtsSlotInts;
}

template <typename CF, typename T, bool AK, bool BK, int E, bool BETA, int VAR = 0>
void launch_pts(const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum, int M, int N, int K,
                int lda, int ldb, int ldc, int ldz, hipStream_t s) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int grid = tiles < num_cus() ? tiles : num_cus();
  int* ctr = nullptr;
  if (pts_dyn() && tiles > grid) ctr = pts_counters(s);
  // non-temporal epilogue stores: bit 0 = C, bit 1 = Z
  int nts = 0;
  switch (pts_nt()) {
    case 1: nts = 3; break;
    case 2: nts = 2; break;
    case 3: nts = (E != kNone) ? 3 : 0; break;
    case 4: nts = (E != kNone) ? 3 : (BETA ? 1 : 0); break;
    case 5: nts = (E != kNone) ? 2 : 0; break;
    default: break;
  }
  static const bool pk = !getenv("PRA_PTS_PK") || atoi(getenv("PRA_PTS_PK")) != 0;
  if (!pk) nts |= 4;  // scalar tanh-GELU' epilogue (packed-f32 form by default)
  gemm_pts_kernel<T, CF, AK, BK, E, BETA, VAR><<<grid, CF::NT, 0, s>>>(
      static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<const uint16_t*>(bias),
      static_cast<uint16_t*>(C), static_cast<uint16_t*>(Z), colsum, M, N, K, lda, ldb, ldc, ldz, ctr, nts);
}

template <typename CF, typename T, bool AK, bool BK>
int launch_pts_e(const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum, int M, int N, int K,
                 int lda, int ldb, int ldc, int ldz, int epi, int beta, hipStream_t s) {
  if (beta && epi != kNone) return -1;
  switch (epi) {
    case kNone:
      if (beta) launch_pts<CF, T, AK, BK, kNone, true>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s);
      else if (CF::NT == 256 && pts_var() == 256)
        launch_pts<CF, T, AK, BK, kNone, false, 256>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s);
      else if (CF::NT == 256 && pts_var() == (256 | (4 << 12)))
        launch_pts<CF, T, AK, BK, kNone, false, 256 | (4 << 12)>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s);
      else if (CF::NT == 256 && pts_var() == (4 << 12))
        launch_pts<CF, T, AK, BK, kNone, false, (4 << 12)>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s);
      else launch_pts<CF, T, AK, BK, kNone, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s);
      return 0;
    case kGeluErf: launch_pts<CF, T, AK, BK, kGeluErf, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s); return 0;
    case kGeluTanh: launch_pts<CF, T, AK, BK, kGeluTanh, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s); return 0;
    case kDGeluErf: launch_pts<CF, T, AK, BK, kDGeluErf, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s); return 0;
    case kDGeluTanh: launch_pts<CF, T, AK, BK, kDGeluTanh, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s); return 0;
    case kGeluErfD:
      if constexpr (AK && !BK) { launch_pts<CF, T, AK, BK, kGeluErfD, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s); return 0; }
      return -1;
    case kGeluTanhD:
      if constexpr (AK && !BK) { launch_pts<CF, T, AK, BK, kGeluTanhD, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s); return 0; }
      return -1;
    case kMulZ:
      if constexpr (AK && BK) { launch_pts<CF, T, AK, BK, kMulZ, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, s); return 0; }
      return -1;
    default: return -1;  // ReLU: the per-tile kernel
  }
}
}  // namespace
}  // namespace pra

// Entry (same contract as pra_gemm_lds with splits = 1, bf16 only). Returns -1 (nothing launched)
// outside what the persistent kernel assumes: K % 128 != 0 or K < 256, beta with an activation,
// a layout this configuration is not built for (LAYOUTS bit mask).
#define PRA_GEMM_PTS_ENTRY(NAME, CFG, LAYOUTS)                                                              \
  extern "C" int NAME(int layout, const void* A, const void* B, const void* bias, void* C, void* Z,            \
                      float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype,       \
                      int epi, int beta, hipStream_t s) {                                                      \
    if (dtype != pra::kBF16 || (K % 128) || K < 256 || !((LAYOUTS >> layout) & 1)) return -1;                 \
    switch (layout) {                                                                                          \
      case 0: if constexpr (LAYOUTS & 1) return pra::launch_pts_e<CFG, pra::bf16, true, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, s); \
              return -1;                                                                                       \
      case 1: if constexpr ((LAYOUTS >> 1) & 1) return pra::launch_pts_e<CFG, pra::bf16, true, true>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, s); \
              return -1;                                                                                       \
      case 2: if constexpr ((LAYOUTS >> 2) & 1) return pra::launch_pts_e<CFG, pra::bf16, false, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, s); \
              return -1;                                                                                       \
      default: return -1;                                                                                      \
    }                                                                                                          \
  }
