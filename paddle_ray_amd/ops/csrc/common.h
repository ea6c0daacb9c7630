// Shared device helpers for the paddle_ray_amd gfx950 kernel library.
// CDNA4: wave64, 16-byte/lane vector accesses, fp32 accumulation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pra {

enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2 };

struct bf16 { uint16_t v; };
using f16 = _Float16;

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
// hardware RNE conversion (v_cvt_pk_bf16_f32 on gfx950; NaN-preserving, branch-free)
typedef float pra_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 pra_b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  pra_f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, pra_b2));
}

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  static __device__ __forceinline__ float to(float x) { return x; }
  static __device__ __forceinline__ float from(float x) { return x; }
};
template <> struct Cvt<bf16> {
  static __device__ __forceinline__ float to(bf16 x) { return bf2f(x.v); }
  static __device__ __forceinline__ bf16 from(float x) { bf16 r; r.v = f2bf(x); return r; }
};
template <> struct Cvt<f16> {
  static __device__ __forceinline__ float to(f16 x) { return (float)x; }
  static __device__ __forceinline__ f16 from(float x) { return (f16)x; }
};

// 8-element vector load/store with fp32 staging (16 B for 2-byte types, 32 B for fp32).
template <typename T> __device__ __forceinline__ void load8(const T* p, float* o);
template <> __device__ __forceinline__ void load8<float>(const float* p, float* o) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <> __device__ __forceinline__ void load8<bf16>(const bf16* p, float* o) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <> __device__ __forceinline__ void load8<f16>(const f16* p, float* o) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  h8 v = *reinterpret_cast<const h8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
}

template <typename T> __device__ __forceinline__ void store8(T* p, const float* o);
template <> __device__ __forceinline__ void store8<float>(float* p, const float* o) {
  *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
}
template <> __device__ __forceinline__ void store8<bf16>(bf16* p, const float* o) {
  uint4 u;
  u.x = pack_bf2(o[0], o[1]);
  u.y = pack_bf2(o[2], o[3]);
  u.z = pack_bf2(o[4], o[5]);
  u.w = pack_bf2(o[6], o[7]);
  *reinterpret_cast<uint4*>(p) = u;
}
template <> __device__ __forceinline__ void store8<f16>(f16* p, const float* o) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  h8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (_Float16)o[i];
  *reinterpret_cast<h8*>(p) = v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide reductions (blockDim.x multiple of 64, <= 1024). `red` needs 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, red[i]);
  return r;
}

#define PRA_DISPATCH_FLOAT(code, T, ...)                 \
  switch (code) {                                         \
    case pra::kF32: { using T = float; __VA_ARGS__; break; } \
    case pra::kF16: { using T = pra::f16; __VA_ARGS__; break; } \
    case pra::kBF16: { using T = pra::bf16; __VA_ARGS__; break; } \
    default: break;                                       \
  }


// erf(u) given e = exp(-u*u) (Abramowitz-Stegun 7.1.26: |error| <= 1.5e-7, far below bf16/f16
// output resolution): one v_rcp + 5 FMAs instead of ocml's erff, and the exp is shared with the
// GELU derivative's exp(-x^2/2) term. Exact-GELU epilogues were VALU-bound on erff.
__device__ __forceinline__ float erf_from_exp(float u, float e) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, fabsf(u), 1.f));
  const float p = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                           0.254829592f);
  return copysignf(1.f - p * e, u);
}
// exact (erf) GELU and its derivative on erf_from_exp
__device__ __forceinline__ float gelu_erf_fast(float x) {
  const float u = x * 0.70710678118654752f;
  return 0.5f * x * (1.f + erf_from_exp(u, __expf(-u * u)));
}
__device__ __forceinline__ float dgelu_erf_fast(float x) {
  const float u = x * 0.70710678118654752f;
  const float e = __expf(-u * u);
  return 0.5f * (1.f + erf_from_exp(u, e)) + x * 0.3989422804014327f * e;
}

}  // namespace pra
