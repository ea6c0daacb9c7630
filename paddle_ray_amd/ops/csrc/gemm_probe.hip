// Diagnostic build of the LDS-DMA MFMA GEMM with per-workgroup phase stamps (PRA_STAMP in
// gemm_core.h): where a tile's time goes (prologue / K loop / epilogue, launch gaps per CU).
// Timing tools only (scripts/gemm_stamps.py); no framework op calls it.
#define PRA_GEMM_STAMPS 1
#include "gemm_core.h"

namespace pra {
namespace {
using PW4 = WCfg<2, 2, 256, 256, true>;
using PW4T = WCfg<2, 2, 256, 256, true, false, false, true>;
using PW4S = WCfg<2, 2, 256, 256, true, true, false, false, true>;     // W4, MUBUF + sc1 DMA
using PW8S = WCfg<2, 4, 256, 256, false, false, false, false, true>;   // W8, sc1 DMA
using PW4TS = WCfg<2, 2, 256, 256, true, true, false, true, true>;     // W4T, MUBUF + sc1 DMA

template <typename CF, bool AK, bool BK>
void probe_launch(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                  unsigned long long* stamps, hipStream_t s) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  gemm_lds_kernel<bf16, CF, AK, BK, kNone, false, false><<<tiles, CF::NT, 0, s>>>(
      static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), nullptr, static_cast<uint16_t*>(C), nullptr,
      nullptr, M, N, K, lda, ldb, ldc, ldc, 1, reinterpret_cast<float*>(stamps));
}
}  // namespace
}  // namespace pra

// cfg: 0 = W8, 1 = W4, 2 = W4T, 3 = W4S, 4 = W8S, 5 = W4TS; layout 0 (x·W) or 1 (dy·Wᵀ).
// stamps: 16 words per workgroup.
// Returns the number of workgroups (or -1).
extern "C" int pra_gemm_probe(int cfg, int layout, const void* A, const void* B, void* C, int M, int N, int K, int lda,
                              int ldb, int ldc, unsigned long long* stamps, hipStream_t s) {
  if (M % 256 || N % 256 || K % 64 || (layout != 0 && layout != 1)) return -1;
  const int tiles = (M / 256) * (N / 256);
  if (layout == 0) {
    switch (cfg) {
      case 0: pra::probe_launch<pra::W8, true, false>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      case 1: pra::probe_launch<pra::PW4, true, false>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      case 2: pra::probe_launch<pra::PW4T, true, false>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      case 3: pra::probe_launch<pra::PW4S, true, false>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      case 4: pra::probe_launch<pra::PW8S, true, false>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      default: pra::probe_launch<pra::PW4TS, true, false>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
    }
  } else {
    switch (cfg) {
      case 0: pra::probe_launch<pra::W8, true, true>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      case 1: pra::probe_launch<pra::PW4, true, true>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      case 2: pra::probe_launch<pra::PW4T, true, true>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      case 3: pra::probe_launch<pra::PW4S, true, true>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      case 4: pra::probe_launch<pra::PW8S, true, true>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
      default: pra::probe_launch<pra::PW4TS, true, true>(A, B, C, M, N, K, lda, ldb, ldc, stamps, s); break;
    }
  }
  return tiles;
}

// Co-residence load for scheduling experiments: nwg workgroups of 256 threads running
// dependent FMA chains on the CUs they land on for `cycles` shader clocks (the stand-in for the
// RCCL channel workgroups that share CUs with the GEMMs during overlapped communication). Every
// wave leaves after at most `cycles` clocks or 1<<24 iterations, whichever comes first.
namespace pra {
namespace {
__global__ void __launch_bounds__(256) spin_hog_k(float* __restrict__ sink, long long cycles) {
  const long long t0 = clock64();
  float a = (float)threadIdx.x, b = 1.0000001f;
  for (int it = 0; it < (1 << 24); ++it) {
#pragma unroll
    for (int u = 0; u < 64; ++u) a = fmaf(a, b, 0.5f);
    if (clock64() - t0 > cycles) break;
  }
  if (a == 12345.f) sink[threadIdx.x] = a;  // keeps the chain alive (never true in practice)
}
}  // namespace
}  // namespace pra

extern "C" void pra_spin_hog(int nwg, long long cycles, float* sink, hipStream_t s) {
  if (nwg > 0) hipLaunchKernelGGL(pra::spin_hog_k, dim3(nwg), dim3(256), 0, s, sink, cycles);
}
