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
// Both operands are staged as they lie in HBM with 16-B stores: A as [m][k] (pitch 72 elements,
// row fragments are ds_read_b128), B as [k][n] (pitch 160 elements); B's column fragments come
// from two ds_read_b64_tr_b16 (hardware-transposed LDS read) each. Both pitches keep every
// 32-lane read phase bank-conflict free. The MFMA is issued as (B-frag, A-frag) so each lane's accumulators hold 4
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
  if (ACT == kGeluErf) return gelu_erf_fast(x);
  if (ACT == kGeluTanh) return 0.5f * x * (1.f + tanhf(0.79788456080286536f * (x + 0.044715f * x * x * x)));
  if (ACT == kRelu) return fmaxf(x, 0.f);
  return x;
}

// Tile configs: <BM, BN, waves along M, waves along N>; each wave owns (BM/WM) x (BN/WN).
template <int BM_, int BN_, int WM_, int WN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NT = 64 * WM_ * WN_;
  static constexpr int TM = BM_ / WM_ / 32, TN = BN_ / WN_ / 32;  // 32x32 MFMA tiles per wave
  static constexpr int LDN = BN_ + 32;                             // 16-dword row skew mod 64 banks
  static constexpr int APASS = BM_ * 8 / NT, BPASS = BN_ * 8 / NT; // 16-B chunks per thread (BK=64)
};
using Small = Cfg<128, 128, 2, 2>;  // 4 waves x 64x64
using Large = Cfg<256, 256, 2, 4>;  // 8 waves x 128x64, 144 KB LDS, 1 workgroup/CU
constexpr int BK = 64, LDK = BK + 8;
typedef short g_v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) g_v4i16 g_lds_v4i16;
typedef uint32_t g_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t g_u32x2 __attribute__((ext_vector_type(2)));

template <typename T, int ACT, typename CF>
__global__ __launch_bounds__(CF::NT) void gemm_bias_act_kernel(const uint16_t* __restrict__ A,
                                                           const uint16_t* __restrict__ B,
                                                           const uint16_t* __restrict__ bias,
                                                           uint16_t* __restrict__ C, uint16_t* __restrict__ Z,
                                                           int M, int N, int K,
                                                           int lda, int ldb, int ldc) {
  constexpr int BM = CF::BM, BN = CF::BN, NT = CF::NT, TM = CF::TM, TN = CF::TN, LDN = CF::LDN;
  constexpr int APASS = CF::APASS, BPASS = CF::BPASS, NCH = BN / 8;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BK * LDN];
  typedef typename G8<T>::type v8;

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nb = gridDim.x;
  int pid = blockIdx.x;
  {  // contiguous tile run per XCD; bijective for any grid (the first r XCDs take q+1 tiles)
    const int q = nb >> 3, r = nb & 7, xcd = pid & 7;
    pid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (pid >> 3);
  }
  const int group = 8 * tiles_n, g = pid / group, first_m = g * 8;
  const int gm = min(tiles_m - first_m, 8);
  const int tm = first_m + (pid % group) % gm, tn = (pid % group) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w / CF::WN, wn = w % CF::WN;
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
      const int c = t + NT * p, kr = c / NCH, nch = c % NCH;
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
      const int c = t + NT * p, kr = c / NCH, nch = c % NCH;
      *reinterpret_cast<uint4*>(&Bs[buf][kr * LDN + nch * 8]) = rb[p];
    }
  };

  g_f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = g_f32x16{};

  const int nk = (K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * BK);
    const uint16_t* as = As[cur] + (wm * TM * 32 + l32) * LDK + h * 8;
    // ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses k-row (base+q), columns
    // 4p..4p+3 of the group's 16 columns, and receives its own column of the 4 rows ->
    // elements k = 16s + 8h + {0..3} (first read) and {4..7} (second read) of column n.
    const int gq = (lane >> 2) & 3, gp = lane & 3, gg = (lane >> 4) & 1;
    const uint16_t* bs = Bs[cur] + (h * 8 + gq) * LDN + wn * TN * 32 + 16 * gg + 4 * gp;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      v8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const v8*>(as + i * 32 * LDK + s * 16);
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const uint16_t* pb = bs + s * 16 * LDN + i * 32;
        const g_v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((g_lds_v4i16*)pb);
        const g_v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((g_lds_v4i16*)(pb + 4 * LDN));
        const g_u32x2 ul = __builtin_bit_cast(g_u32x2, lo), uh = __builtin_bit_cast(g_u32x2, hi);
        const g_u32x4 u = {ul[0], ul[1], uh[0], uh[1]};
        bf[i] = __builtin_bit_cast(v8, u);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = gmma<T>(bf[j], af[i], acc[i][j]);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  // epilogue: acc[i][j][r] = C[m = m0+(wm*TM+i)*32+l32][n = n0+(wn*TN+j)*32 + (r&3) + 8*(r>>2) + 4*h]
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + (wm * TM + i) * 32 + l32;
    if (m >= M) continue;
    uint16_t* crow = C + (int64_t)m * ldc;
    uint16_t* zrow = Z ? Z + (int64_t)m * ldc : nullptr;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + (wn * TN + j) * 32 + 8 * q + 4 * h;
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

template <typename T, typename CF>
void launch_cfg(const uint16_t* pa, const uint16_t* pb, const uint16_t* pbias, uint16_t* pc, uint16_t* pz, int M,
                int N, int K, int lda, int ldb, int ldc, int a, hipStream_t s) {
  const int tiles = ((M + CF::BM - 1) / CF::BM) * ((N + CF::BN - 1) / CF::BN);
  switch (a) {
    case kGeluErf: gemm_bias_act_kernel<T, kGeluErf, CF><<<tiles, CF::NT, 0, s>>>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc); break;
    case kGeluTanh: gemm_bias_act_kernel<T, kGeluTanh, CF><<<tiles, CF::NT, 0, s>>>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc); break;
    case kRelu: gemm_bias_act_kernel<T, kRelu, CF><<<tiles, CF::NT, 0, s>>>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc); break;
    default: gemm_bias_act_kernel<T, kNone, CF><<<tiles, CF::NT, 0, s>>>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc); break;
  }
}

// Large tiles (1 workgroup/CU) once there are >= 3 rounds of them over the 256 CUs, or 2 rounds
// with a long K loop; small otherwise. Measured at M=16384, N=2048 (512 large tiles):
// K=2048 large 222 us vs small 201 us; K=8192 large 634 us vs small 672 us.
template <typename T>
void launch(const void* A, const void* B, const void* bias, void* C, void* Z, int M, int N, int K, int lda, int ldb,
            int ldc, int a, hipStream_t s) {
  const auto* pa = static_cast<const uint16_t*>(A);
  const auto* pb = static_cast<const uint16_t*>(B);
  const auto* pbias = static_cast<const uint16_t*>(bias);
  auto* pc = static_cast<uint16_t*>(C);
  auto* pz = static_cast<uint16_t*>(Z);
  const int64_t big = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  if (big >= 768 || (big >= 512 && K >= 4096)) launch_cfg<T, Large>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc, a, s);
  else launch_cfg<T, Small>(pa, pb, pbias, pc, pz, M, N, K, lda, ldb, ldc, a, s);
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
