// MFMA GEMM with fused epilogue for gfx950 (CDNA4):
//   C[M,N] = act(A[M,K] @ B[K,N] + bias[N])     A, B, C row-major, bf16/f16 in and out, fp32 accum.
// B is in Paddle's Linear layout ([in, out], reference python/paddle/nn/functional/common.py:1843
// `linear` -> matmul(x, weight) + bias; fused variant paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue
// -> cublasLt epilogue BIAS/GELU/RELU). Here the epilogue runs in registers on the MFMA accumulators,
// so the activation never makes an extra HBM round trip.
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 wave64s in 2x2, each wave owns 64x64 =
// 2x2 v_mfma_f32_32x32x16 accumulators), K staged 64 at a time through double-buffered LDS (one
// barrier per K tile; the next tile's global loads are issued before the current tile's MFMAs).
// A is staged row-major [m][k]; B is transposed on its way into LDS ([n][k]) so both operand
// fragments are single 16-B ds_read_b128s. Row pitch 72 elements (144 B) keeps the fragment reads
// bank-conflict free. The MFMA is issued as (B-frag, A-frag) so each lane's accumulators hold 4
// consecutive output columns -> packed 8-B stores in the epilogue.
//
// Tile order: workgroups are dispatched round-robin over the 8 XCDs; the linear id is remapped so
// each XCD gets a contiguous run of tiles, then grouped 8 M-tiles at a time so neighbouring
// tiles share A/B panels inside one XCD's L2.
#include "common.h"

namespace pra {
namespace {

typedef float g_f32x16 __attribute__((ext_vector_type(16)));
template <typename T> struct G8;
template <> struct G8<bf16> { typedef __bf16 type __attribute__((ext_vector_type(8))); };
template <> struct G8<f16> { typedef _Float16 type __attribute__((ext_vector_type(8))); };

template <typename T>
__device__ __forceinline__ g_f32x16 gmma(typename G8<T>::type a, typename G8<T>::type b, g_f32x16 c);
template <>
__device__ __forceinline__ g_f32x16 gmma<bf16>(G8<bf16>::type a, G8<bf16>::type b, g_f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ g_f32x16 gmma<f16>(G8<f16>::type a, G8<f16>::type b, g_f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <typename T> __device__ __forceinline__ float g_to(uint16_t u);
template <> __device__ __forceinline__ float g_to<bf16>(uint16_t u) { return bf2f(u); }
template <> __device__ __forceinline__ float g_to<f16>(uint16_t u) { return (float)__builtin_bit_cast(_Float16, u); }
template <typename T> __device__ __forceinline__ uint32_t g_pack(float a, float b);
template <> __device__ __forceinline__ uint32_t g_pack<bf16>(float a, float b) { return pack_bf2(a, b); }
template <> __device__ __forceinline__ uint32_t g_pack<f16>(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)b) << 16);
}

enum Act : int { kNone = 0, kGeluErf = 1, kGeluTanh = 2, kRelu = 3 };

template <int ACT>
__device__ __forceinline__ float act(float x) {
  if (ACT == kGeluErf) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  if (ACT == kGeluTanh) return 0.5f * x * (1.f + tanhf(0.79788456080286536f * (x + 0.044715f * x * x * x)));
  if (ACT == kRelu) return fmaxf(x, 0.f);
  return x;
}

constexpr int BM = 128, BN = 128, BK = 64, LDK = BK + 8, NT = 256;
constexpr int APASS = BM * BK / 8 / NT;  // 16-B chunks per thread per K tile (A)
constexpr int BPASS = BN * BK / 8 / NT;  // (B)

template <typename T, int ACT>
__global__ __launch_bounds__(NT) void gemm_bias_act_kernel(const uint16_t* __restrict__ A,
                                                           const uint16_t* __restrict__ B,
                                                           const uint16_t* __restrict__ bias,
                                                           uint16_t* __restrict__ C, uint16_t* __restrict__ Z,
                                                           int M, int N, int K,
                                                           int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) uint16_t As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BN * LDK];
  typedef typename G8<T>::type v8;

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nb = gridDim.x;
  int pid = blockIdx.x;
  if ((nb & 7) == 0) pid = (pid & 7) * (nb >> 3) + (pid >> 3);  // contiguous tile run per XCD
  const int group = 8 * tiles_n, g = pid / group, first_m = g * 8;
  const int gm = min(tiles_m - first_m, 8);
  const int tm = first_m + (pid % group) % gm, tn = (pid % group) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int l32 = lane & 31, h = lane >> 5;

  uint4 ra[APASS], rb[BPASS];
  auto load = [&](int k0) {
#pragma unroll
    for (int p = 0; p < APASS; ++p) {
      const int c = t + NT * p, row = c >> 3, ch = c & 7;
      const int gmr = m0 + row, gk = k0 + ch * 8;
      ra[p] = (gmr < M && gk < K) ? *reinterpret_cast<const uint4*>(A + (int64_t)gmr * lda + gk)
                                  : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < BPASS; ++p) {
      const int c = t + NT * p, kr = c & (BK - 1), nch = c / BK;  // lanes of a wave walk k
      const int gk = k0 + kr, gn = n0 + nch * 8;
      rb[p] = (gk < K && gn < N) ? *reinterpret_cast<const uint4*>(B + (int64_t)gk * ldb + gn)
                                 : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int p = 0; p < APASS; ++p) {
      const int c = t + NT * p, row = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(&As[buf][row * LDK + ch * 8]) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < BPASS; ++p) {
      const int c = t + NT * p, kr = c & (BK - 1), nch = c / BK;
      uint16_t* dst = &Bs[buf][(nch * 8) * LDK + kr];
      const uint32_t wv[4] = {rb[p].x, rb[p].y, rb[p].z, rb[p].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dst[(2 * i) * LDK] = (uint16_t)(wv[i] & 0xffff);
        dst[(2 * i + 1) * LDK] = (uint16_t)(wv[i] >> 16);
      }
    }
  };

  g_f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = g_f32x16{};

  const int nk = (K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * BK);
    const uint16_t* as = As[cur] + (wm * 64 + l32) * LDK + h * 8;
    const uint16_t* bs = Bs[cur] + (wn * 64 + l32) * LDK + h * 8;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      v8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = *reinterpret_cast<const v8*>(as + i * 32 * LDK + s * 16);
        bf[i] = *reinterpret_cast<const v8*>(bs + i * 32 * LDK + s * 16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = gmma<T>(bf[j], af[i], acc[i][j]);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  // epilogue: acc[i][j][r] = C[m = m0+wm*64+i*32+l32][n = n0+wn*64+j*32 + (r&3) + 8*(r>>2) + 4*h]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 64 + i * 32 + l32;
    if (m >= M) continue;
    uint16_t* crow = C + (int64_t)m * ldc;
    uint16_t* zrow = Z ? Z + (int64_t)m * ldc : nullptr;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + wn * 64 + j * 32 + 8 * q + 4 * h;
        if (n >= N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
        if (bias) {
          const uint2 bb = *reinterpret_cast<const uint2*>(bias + n);
          v[0] += g_to<T>(bb.x & 0xffff); v[1] += g_to<T>(bb.x >> 16);
          v[2] += g_to<T>(bb.y & 0xffff); v[3] += g_to<T>(bb.y >> 16);
        }
        uint2 o;
        if (ACT != kNone && zrow) {  // pre-activation for the backward pass
          o.x = g_pack<T>(v[0], v[1]);
          o.y = g_pack<T>(v[2], v[3]);
          *reinterpret_cast<uint2*>(zrow + n) = o;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = act<ACT>(v[e]);
        o.x = g_pack<T>(v[0], v[1]);
        o.y = g_pack<T>(v[2], v[3]);
        *reinterpret_cast<uint2*>(crow + n) = o;
      }
    }
  }
}

template <typename T>
void launch(const void* A, const void* B, const void* bias, void* C, void* Z, int M, int N, int K, int lda, int ldb,
            int ldc, int a, hipStream_t s) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const auto* pa = static_cast<const uint16_t*>(A);
  const auto* pb = static_cast<const uint16_t*>(B);
  const auto* pbias = static_cast<const uint16_t*>(bias);
  auto* pc = static_cast<uint16_t*>(C);
  auto* pz = static_cast<uint16_t*>(Z);
  switch (a) {
    case kGeluErf: gemm_bias_act_kernel<T, kGeluErf><<<tiles, NT, 0, s>>>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc); break;
    case kGeluTanh: gemm_bias_act_kernel<T, kGeluTanh><<<tiles, NT, 0, s>>>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc); break;
    case kRelu: gemm_bias_act_kernel<T, kRelu><<<tiles, NT, 0, s>>>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc); break;
    default: gemm_bias_act_kernel<T, kNone><<<tiles, NT, 0, s>>>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc); break;
  }
}

}  // namespace
}  // namespace pra

// Returns 0 on launch, -1 if the shape/layout is outside what the kernel assumes (caller falls
// back loudly). Z (optional, ldc pitch) receives act's input when act != none: 16-B aligned rows (K, N, lda, ldb, ldc multiples of 8), 2-byte dtypes only.
extern "C" int pra_gemm_bias_act(const void* A, const void* B, const void* bias, void* C, void* Z, int M, int N, int K,
                                 int lda, int ldb, int ldc, int dtype, int act, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return -1;
  if ((K & 7) || (N & 7) || (lda & 7) || (ldb & 7) || (ldc & 7) || lda < K || ldb < N || ldc < N) return -1;
  if (act < 0 || act > 3) return -1;
  if (dtype == pra::kBF16) pra::launch<pra::bf16>(A, B, bias, C, Z, M, N, K, lda, ldb, ldc, act, s);
  else if (dtype == pra::kF16) pra::launch<pra::f16>(A, B, bias, C, Z, M, N, K, lda, ldb, ldc, act, s);
  else return -1;
  return 0;
}
