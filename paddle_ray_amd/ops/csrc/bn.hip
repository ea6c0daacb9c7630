// BatchNorm (+ residual add + ReLU) for channels-last activations on gfx950.
//
// Parity: paddle/phi/kernels/gpu/batch_norm_kernel.cu, batch_norm_grad_kernel.cu and the
// fused variants paddle/fluid/operators/fused/fused_bn_activation_op.cu,
// fused_bn_add_activation_op.cu (y = act(BN(x) + z)).
//
// x is viewed as [M, C] (M = N*H*W, NHWC) with C % 8 == 0, so one lane owns 8 channels and
// every access is a 16-byte vector. Training forward = 3 launches:
//   bn_reduce_k   (MODE 0)  per-row-block partial sums of (x - K) and (x - K)^2, where K is
//                           row 0 of x (shifted-data variance: no E[x^2]-E[x]^2 cancellation)
//   bn_fin_fwd_k            per channel: merge partials in fp64 -> mean, invstd, running
//                           stats update (paddle momentum convention), scale/shift
//   bn_apply_k              y = act(x * scale + shift [+ z])
// Backward = 3 launches with the same shape:
//   bn_reduce_k   (MODE 1)  partial sums of g and g * (x - mean), g = dy masked by y > 0
//   bn_fin_bwd_k            dscale, dbias, and the per-channel dx coefficients
//   bn_bwd_apply_k          dx = a*g + c1*x + c0 (+ dz = g)
// The row-block partials are written once and merged deterministically (no float atomics).
#include "common.h"

namespace pra {

constexpr int kBnThreads = 256;   // elementwise apply kernels
constexpr int kRedThreads = 1024; // reduction kernels: 16 waves, up to 128 rows per pass

__device__ __forceinline__ float ldw(const void* p, int i, int dt) {
  if (dt == kF32) return ((const float*)p)[i];
  if (dt == kBF16) return bf2f(((const uint16_t*)p)[i]);
  return (float)((const f16*)p)[i];
}
__device__ __forceinline__ void stw(void* p, int i, int dt, float v) {
  if (dt == kF32) ((float*)p)[i] = v;
  else if (dt == kBF16) ((uint16_t*)p)[i] = f2bf(v);
  else ((f16*)p)[i] = (f16)v;
}

// Per-row gradient g for the backward reductions: dy masked by the forward ReLU, read either
// from the 1-bit-per-element mask the forward wrote (1 B per 8 channels) or from y.
template <typename T, bool RELU>
__device__ __forceinline__ void load_g(const T* __restrict__ dy, const T* __restrict__ y,
                                       const uint8_t* __restrict__ mask, size_t r, int C, int cv, float* g) {
  load8<T>(dy + r * C + cv * 8, g);
  if (RELU) {
    if (mask) {
      const uint32_t m = mask[r * (C >> 3) + cv];
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = (m >> i) & 1u ? g[i] : 0.f;
    } else {
      float yv[8];
      load8<T>(y + r * C + cv * 8, yv);
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
    }
  }
}

// Block = RPI row lanes x CVB vector-columns (CVB = min(C/8, 64), RPI = 1024/CVB); grid =
// (C/8/CVB, nrb). Each lane keeps 4 rows of loads in flight.
// MODE 0: s1 = sum(x - K), s2 = sum((x - K)^2), K = x[0, c]
// MODE 1: s1 = sum(g),     s2 = sum(g * (x - mean[c]))
template <typename T, int MODE, bool RELU>
__global__ void __launch_bounds__(kRedThreads) bn_reduce_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                           const T* __restrict__ y, const uint8_t* __restrict__ mask,
                                                           const float* __restrict__ mean, float* __restrict__ part,
                                                           int M, int C, int rpb) {
  __shared__ float red[8 * kRedThreads];
  const int CV = C >> 3;
  const int cvb = CV < 64 ? CV : 64;
  const int rpi = kRedThreads / cvb;
  const int tid = threadIdx.x, cl = tid % cvb, rl = tid / cvb;
  const int cv = blockIdx.x * cvb + cl;
  const bool active = rl < rpi && cv < CV;
  const int r0 = blockIdx.y * rpb;
  const int r1 = min(M, r0 + rpb);
  float K[8], s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s1[i] = 0.f; s2[i] = 0.f; K[i] = 0.f; }
  if (active) {
    if (MODE == 0) {
      load8<T>(x + cv * 8, K);
    } else {
      const float4 m0 = *reinterpret_cast<const float4*>(mean + cv * 8);
      const float4 m1 = *reinterpret_cast<const float4*>(mean + cv * 8 + 4);
      K[0] = m0.x; K[1] = m0.y; K[2] = m0.z; K[3] = m0.w; K[4] = m1.x; K[5] = m1.y; K[6] = m1.z; K[7] = m1.w;
    }
    int r = r0 + rl;
    for (; r + 3 * rpi < r1; r += 4 * rpi) {
      float a[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load8<T>(x + (size_t)(r + u * rpi) * C + cv * 8, a[u]);
      if (MODE == 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 8; ++i) { float d = a[u][i] - K[i]; s1[i] += d; s2[i] += d * d; }
      } else {
        float g[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) load_g<T, RELU>(dy, y, mask, (size_t)(r + u * rpi), C, cv, g[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 8; ++i) { s1[i] += g[u][i]; s2[i] += g[u][i] * (a[u][i] - K[i]); }
      }
    }
    for (; r < r1; r += rpi) {
      float a[8];
      load8<T>(x + (size_t)r * C + cv * 8, a);
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) { float d = a[i] - K[i]; s1[i] += d; s2[i] += d * d; }
      } else {
        float g[8];
        load_g<T, RELU>(dy, y, mask, (size_t)r, C, cv, g);
#pragma unroll
        for (int i = 0; i < 8; ++i) { s1[i] += g[i]; s2[i] += g[i] * (a[i] - K[i]); }
      }
    }
  }
  // cross-row-lane reduction through LDS ([k][tid] layout: consecutive cl, consecutive banks);
  // s1 then s2 through the same 32 KB, a halving tree when rpi is a power of two
  const bool pow2 = (rpi & (rpi - 1)) == 0 && rpi * cvb == kRedThreads;
  float* outp[2] = {part + (size_t)blockIdx.y * C, part + ((size_t)gridDim.y + blockIdx.y) * C};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float* sv = h == 0 ? s1 : s2;
#pragma unroll
    for (int i = 0; i < 8; ++i) red[i * kRedThreads + tid] = sv[i];
    __syncthreads();
    if (pow2) {
      for (int st = rpi >> 1; st > 0; st >>= 1) {
        if (rl < st) {
#pragma unroll
          for (int i = 0; i < 8; ++i) red[i * kRedThreads + tid] += red[i * kRedThreads + tid + st * cvb];
        }
        __syncthreads();
      }
    } else if (rl == 0) {
      for (int j = 1; j < rpi; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) red[i * kRedThreads + tid] += red[i * kRedThreads + j * cvb + cl];
    }
    if (rl == 0 && cv < CV) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = red[i * kRedThreads + tid];
      *reinterpret_cast<float4*>(outp[h] + cv * 8) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(outp[h] + cv * 8 + 4) = make_float4(o[4], o[5], o[6], o[7]);
    }
    __syncthreads();
  }
}

// Merge nrb partial rows for 64 channels per block: 16 row lanes x 64 channels, fp64 sums.
__device__ __forceinline__ void merge_parts(const float* __restrict__ part, int nrb, int C, int c, int rl, double& S1,
                                            double& S2, double* red) {
  double a = 0.0, b = 0.0;
  if (c < C) {
    // 16 loads in flight per lane (the conv-epilogue statistics arrive as up to ~1600 tile rows;
    // one dependent load per row made the merge latency-bound); same summation order as a plain loop
    const float* p1 = part + c;
    const float* p2 = part + (size_t)nrb * C + c;
    int j = rl;
    for (; j + 16 * 7 < nrb; j += 16 * 8) {
      float u[8], v[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) { u[t] = p1[(size_t)(j + 16 * t) * C]; v[t] = p2[(size_t)(j + 16 * t) * C]; }
#pragma unroll
      for (int t = 0; t < 8; ++t) { a += u[t]; b += v[t]; }
    }
    for (; j < nrb; j += 16) {
      a += p1[(size_t)j * C];
      b += p2[(size_t)j * C];
    }
  }
  red[threadIdx.x] = a;
  red[1024 + threadIdx.x] = b;
  __syncthreads();
  S1 = 0.0; S2 = 0.0;
  if (rl == 0) {
    for (int j = 0; j < 16; ++j) { S1 += red[j * 64 + (threadIdx.x & 63)]; S2 += red[1024 + j * 64 + (threadIdx.x & 63)]; }
  }
}

// Partial-row pre-merge for the statistics a convolution epilogue produced (one row per output
// tile: up to ~6300 rows for the ResNet stem), so the finalize's single block per 64 channels
// does not walk thousands of rows: [2][nrb][C] -> [2][ceil(nrb/64)][C], block (c64, r) sums rows
// 64r .. 64r+63 (16 row lanes x 4 rows, fixed order: deterministic).
__global__ void __launch_bounds__(1024) bn_premerge_k(const float* __restrict__ part, float* __restrict__ out,
                                                      int nrb, int nrb2, int C) {
  __shared__ float red[2][1024];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6, r0 = blockIdx.y * 64;
  float a = 0.f, b = 0.f;
  if (c < C) {
    float u[4], v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = r0 + rl + 16 * t;
      u[t] = j < nrb ? part[(size_t)j * C + c] : 0.f;
      v[t] = j < nrb ? part[((size_t)nrb + j) * C + c] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) { a += u[t]; b += v[t]; }
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  if (rl == 0 && c < C) {
    float sa = 0.f, sb = 0.f;
    for (int j = 0; j < 16; ++j) { sa += red[0][j * 64 + threadIdx.x]; sb += red[1][j * 64 + threadIdx.x]; }
    out[(size_t)blockIdx.y * C + c] = sa;
    out[((size_t)nrb2 + blockIdx.y) * C + c] = sb;
  }
}

// out: mean[C], invstd[C] (saved for backward), coef[0:C] = scale, coef[C:2C] = shift.
template <typename T>
__global__ void __launch_bounds__(1024) bn_fin_fwd_k(const float* __restrict__ part, const T* __restrict__ x,
                                                     const void* __restrict__ w, const void* __restrict__ b, int dtw,
                                                     float* __restrict__ rmean, float* __restrict__ rvar,
                                                     float* __restrict__ mean, float* __restrict__ invstd,
                                                     float* __restrict__ coef, int nrb, int M, int C, float eps,
                                                     float momentum, const float* __restrict__ kshift = nullptr) {
  __shared__ double red[2048];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  double S1, S2;
  merge_parts(part, nrb, C, c, rl, S1, S2, red);
  if (rl != 0 || c >= C) return;
  // the shift the partial sums were taken around: row 0 of x (bn_reduce_k) or, for statistics
  // produced by a convolution epilogue, the running mean it was given
  const double K = kshift ? (double)kshift[c] : (double)Cvt<T>::to(x[c]);
  const double d = S1 / M;
  double var = S2 / M - d * d;
  if (var < 0.0) var = 0.0;
  const float mu = (float)(K + d);
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  mean[c] = mu;
  invstd[c] = is;
  const float sc = (w ? ldw(w, c, dtw) : 1.f) * is;
  coef[c] = sc;
  coef[C + c] = (b ? ldw(b, c, dtw) : 0.f) - mu * sc;
  if (rmean) {
    const float uvar = M > 1 ? (float)(var * M / (M - 1)) : (float)var;
    rmean[c] = momentum * rmean[c] + (1.f - momentum) * mu;
    rvar[c] = momentum * rvar[c] + (1.f - momentum) * uvar;
  }
}

// inference: scale/shift from running statistics
__global__ void bn_fin_infer_k(const void* __restrict__ w, const void* __restrict__ b, int dtw,
                               const float* __restrict__ rmean, const float* __restrict__ rvar,
                               float* __restrict__ coef, int C, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = rsqrtf(rvar[c] + eps);
  const float sc = (w ? ldw(w, c, dtw) : 1.f) * is;
  coef[c] = sc;
  coef[C + c] = (b ? ldw(b, c, dtw) : 0.f) - rmean[c] * sc;
}

// dscale = S2 * invstd, dbias = S1;  dx = a*g + c1*x + c0 with
//   a = w*invstd, c1 = -a*invstd^2*S2/M, c0 = -a*S1/M - c1*mean.  coef = [a | c1 | c0]
__global__ void __launch_bounds__(1024) bn_fin_bwd_k(const float* __restrict__ part, const void* __restrict__ w,
                                                     int dtw, const float* __restrict__ mean,
                                                     const float* __restrict__ invstd, void* __restrict__ dw,
                                                     void* __restrict__ db, float* __restrict__ coef, int nrb, int M,
                                                     int C, int acc) {
  __shared__ double red[2048];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  double S1, S2;
  merge_parts(part, nrb, C, c, rl, S1, S2, red);
  if (rl != 0 || c >= C) return;
  const float is = invstd[c];
  // acc: add into the existing parameter gradients (no separate AccumulateGrad add)
  if (dw) stw(dw, c, dtw, (float)(S2 * is) + (acc ? ldw(dw, c, dtw) : 0.f));
  if (db) stw(db, c, dtw, (float)S1 + (acc ? ldw(db, c, dtw) : 0.f));
  const float a = (w ? ldw(w, c, dtw) : 1.f) * is;
  const float c1 = (float)(-(double)a * is * is * S2 / M);
  coef[c] = a;
  coef[C + c] = c1;
  coef[2 * C + c] = (float)(-(double)a * S1 / M) - c1 * mean[c];
}

__device__ __forceinline__ void ld8f(const float* p, float* o) {
  const float4 u = *reinterpret_cast<const float4*>(p);
  const float4 v = *reinterpret_cast<const float4*>(p + 4);
  o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w; o[4] = v.x; o[5] = v.y; o[6] = v.z; o[7] = v.w;
}

// y = act(x * scale + shift [+ z]); grid-stride over 8-element vectors, two vectors (v and
// v + stride) in flight per lane, channel tracked incrementally instead of a per-vector modulo.
// With RELU and a mask pointer, also writes the ReLU keep-bits (1 B per vector) for backward.
template <typename T, bool RELU, bool RES>
__device__ __forceinline__ void bn_apply_one(const T* __restrict__ x, const T* __restrict__ z,
                                             const float* __restrict__ coef, T* __restrict__ y,
                                             uint8_t* __restrict__ mask, uint32_t v, uint32_t cv, int C) {
  float a[8], sc[8], sh[8], r[8];
  load8<T>(x + (size_t)v * 8, a);
  if (RES) load8<T>(z + (size_t)v * 8, r);
  ld8f(coef + cv * 8, sc);
  ld8f(coef + C + cv * 8, sh);
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float o = a[i] * sc[i] + sh[i];
    if (RES) o += r[i];
    if (RELU) { bits |= (o > 0.f ? 1u : 0u) << i; o = fmaxf(o, 0.f); }
    a[i] = o;
  }
  store8<T>(y + (size_t)v * 8, a);
  if (RELU && mask) mask[v] = (uint8_t)bits;
}

template <typename T, bool RELU, bool RES>
__global__ void __launch_bounds__(kBnThreads) bn_apply_k(const T* __restrict__ x, const T* __restrict__ z,
                                                         const float* __restrict__ coef, T* __restrict__ y,
                                                         uint8_t* __restrict__ mask, uint32_t nvec, int C) {
  const uint32_t CV = C >> 3;
  const uint32_t stride = gridDim.x * kBnThreads;
  uint32_t v = blockIdx.x * kBnThreads + threadIdx.x;
  if (v >= nvec) return;
  const uint32_t step = stride % CV;
  uint32_t cv = v % CV;
  for (; v < nvec; v += 2 * stride) {
    uint32_t cv2 = cv + step;
    if (cv2 >= CV) cv2 -= CV;
    bn_apply_one<T, RELU, RES>(x, z, coef, y, mask, v, cv, C);
    if (v + stride < nvec) bn_apply_one<T, RELU, RES>(x, z, coef, y, mask, v + stride, cv2, C);
    cv = cv2 + step;
    if (cv >= CV) cv -= CV;
  }
}

template <typename T, bool RELU>
__device__ __forceinline__ void bn_bwd_one(const T* __restrict__ dy, const T* __restrict__ y,
                                           const uint8_t* __restrict__ mask, const T* __restrict__ x,
                                           const float* __restrict__ coef, T* __restrict__ dx, T* __restrict__ dz,
                                           uint32_t v, uint32_t cv, int C) {
  float g[8], xv[8], a[8], c1[8], c0[8];
  load_g<T, RELU>(dy, y, mask, v, 8, 0, g);  // row v of an [nvec, 8] view
  load8<T>(x + (size_t)v * 8, xv);
  ld8f(coef + cv * 8, a);
  ld8f(coef + C + cv * 8, c1);
  ld8f(coef + 2 * C + cv * 8, c0);
  if (dz) store8<T>(dz + (size_t)v * 8, g);
#pragma unroll
  for (int i = 0; i < 8; ++i) xv[i] = a[i] * g[i] + c1[i] * xv[i] + c0[i];
  store8<T>(dx + (size_t)v * 8, xv);
}

template <typename T, bool RELU>
__global__ void __launch_bounds__(kBnThreads) bn_bwd_apply_k(const T* __restrict__ dy, const T* __restrict__ y,
                                                             const uint8_t* __restrict__ mask,
                                                             const T* __restrict__ x, const float* __restrict__ coef,
                                                             T* __restrict__ dx, T* __restrict__ dz, uint32_t nvec,
                                                             int C) {
  const uint32_t CV = C >> 3;
  const uint32_t stride = gridDim.x * kBnThreads;
  uint32_t v = blockIdx.x * kBnThreads + threadIdx.x;
  if (v >= nvec) return;
  const uint32_t step = stride % CV;
  uint32_t cv = v % CV;
  for (; v < nvec; v += 2 * stride) {
    uint32_t cv2 = cv + step;
    if (cv2 >= CV) cv2 -= CV;
    bn_bwd_one<T, RELU>(dy, y, mask, x, coef, dx, dz, v, cv, C);
    if (v + stride < nvec) bn_bwd_one<T, RELU>(dy, y, mask, x, coef, dx, dz, v + stride, cv2, C);
    cv = cv2 + step;
    if (cv >= CV) cv -= CV;
  }
}

static inline int bn_grid_x(int C) {
  const int CV = C / 8, cvb = CV < 64 ? CV : 64;
  return (CV + cvb - 1) / cvb;
}
static inline int bn_rpi(int C) {
  const int CV = C / 8, cvb = CV < 64 ? CV : 64;
  return kRedThreads / cvb;
}
static inline int bn_rpb(int M, int C, int nrb) {
  const int rpi = bn_rpi(C);
  int rpb = (M + nrb - 1) / nrb;
  return (rpb + rpi - 1) / rpi * rpi;
}
static inline unsigned bn_apply_grid(uint32_t nvec) {
  // 256 CUs x 8 resident 256-thread blocks, two vectors per lane per pass
  unsigned g = (nvec / 2 + kBnThreads - 1) / kBnThreads;
  return g < 2048u ? (g ? g : 1u) : 2048u;
}

template <typename T>
static void launch_apply(const void* x, const void* z, const float* coef, void* y, uint8_t* mask, uint32_t nvec, int C,
                         int relu, hipStream_t s) {
  const unsigned g = bn_apply_grid(nvec);
  if (relu && z)
    hipLaunchKernelGGL((bn_apply_k<T, true, true>), dim3(g), dim3(kBnThreads), 0, s, (const T*)x, (const T*)z, coef,
                       (T*)y, mask, nvec, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_k<T, true, false>), dim3(g), dim3(kBnThreads), 0, s, (const T*)x, nullptr, coef,
                       (T*)y, mask, nvec, C);
  else if (z)
    hipLaunchKernelGGL((bn_apply_k<T, false, true>), dim3(g), dim3(kBnThreads), 0, s, (const T*)x, (const T*)z, coef,
                       (T*)y, nullptr, nvec, C);
  else
    hipLaunchKernelGGL((bn_apply_k<T, false, false>), dim3(g), dim3(kBnThreads), 0, s, (const T*)x, nullptr, coef,
                       (T*)y, nullptr, nvec, C);
}

}  // namespace pra

using namespace pra;

extern "C" {
// Row-block count of the reductions: ~512 blocks of 1024 threads (2 per CU), at most 256
// partial rows so the per-channel merge stays a few microseconds.
int pra_bn_nrb(int M, int C) {
  if (C % 8 != 0 || M <= 0) return 0;
  const int gx = bn_grid_x(C);
  int nrb = (512 + gx - 1) / gx;
  if (nrb > 256) nrb = 256;
  const int rpi = bn_rpi(C);
  const int maxr = (M + 4 * rpi - 1) / (4 * rpi);  // >= 4 rows per lane
  if (nrb > maxr) nrb = maxr;
  if (nrb < 1) nrb = 1;
  // the effective count after rounding rows-per-block up to the row-lane count
  const int rpb = bn_rpb(M, C, nrb);
  return (M + rpb - 1) / rpb;
}

// part: [2, nrb, C] fp32 scratch; coef: [2, C] fp32 scratch (scale | shift); mask (optional,
// relu only): [M*C/8] bytes of ReLU keep-bits for the backward.
void pra_bn_fwd_train(const void* x, const void* z, const void* w, const void* b, float* rmean, float* rvar, void* y,
                      uint8_t* mask, float* mean, float* invstd, float* part, float* coef, int M, int C, int nrb,
                      float eps, float momentum, int relu, int dt, int dtw, hipStream_t s) {
  const int rpb = bn_rpb(M, C, nrb);
  const dim3 rg(bn_grid_x(C), nrb);
  const uint32_t nvec = (uint32_t)((size_t)M * C / 8);
  PRA_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL((bn_reduce_k<T, 0, false>), rg, dim3(kRedThreads), 0, s, (const T*)x, nullptr, nullptr,
                       nullptr, nullptr, part, M, C, rpb);
    hipLaunchKernelGGL((bn_fin_fwd_k<T>), dim3((C + 63) / 64), dim3(1024), 0, s, part, (const T*)x, w, b, dtw, rmean,
                       rvar, mean, invstd, coef, nrb, M, C, eps, momentum, (const float*)nullptr);
    launch_apply<T>(x, z, coef, y, mask, nvec, C, relu, s);
  });
}

// Forward from statistics produced elsewhere (the implicit-GEMM convolution's epilogue): part
// [2][nrb][C] = per-row-block sums of (x - kshift) and (x - kshift)^2; then finalize + apply.
void pra_bn_fwd_parts(const void* x, const void* z, const void* w, const void* b, float* rmean, float* rvar, void* y,
                      uint8_t* mask, float* mean, float* invstd, const float* part, const float* kshift, float* coef,
                      int M, int C, int nrb, float eps, float momentum, int relu, int dt, int dtw, hipStream_t s) {
  const uint32_t nvec = (uint32_t)((size_t)M * C / 8);
  PRA_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL((bn_fin_fwd_k<T>), dim3((C + 63) / 64), dim3(1024), 0, s, part, (const T*)x, w, b, dtw, rmean,
                       rvar, mean, invstd, coef, nrb, M, C, eps, momentum, kshift);
    launch_apply<T>(x, z, coef, y, mask, nvec, C, relu, s);
  });
}

// out [2][ceil(nrb/64)][C] (see bn_premerge_k)
void pra_bn_premerge(const float* part, float* out, int nrb, int C, hipStream_t s) {
  const int nrb2 = (nrb + 63) / 64;
  hipLaunchKernelGGL(bn_premerge_k, dim3((C + 63) / 64, nrb2), dim3(1024), 0, s, part, out, nrb, nrb2, C);
}

void pra_bn_fwd_infer(const void* x, const void* z, const void* w, const void* b, const float* rmean,
                      const float* rvar, void* y, float* coef, int M, int C, float eps, int relu, int dt, int dtw,
                      hipStream_t s) {
  hipLaunchKernelGGL(bn_fin_infer_k, dim3((C + 255) / 256), dim3(256), 0, s, w, b, dtw, rmean, rvar, coef, C, eps);
  const uint32_t nvec = (uint32_t)((size_t)M * C / 8);
  PRA_DISPATCH_FLOAT(dt, T, launch_apply<T>(x, z, coef, y, nullptr, nvec, C, relu, s));
}

// relu: the keep-mask comes from `mask` (if non-null) else from the forward OUTPUT y.
// dz (residual grad) may be null. coef: [3, C] fp32 scratch.
void pra_bn_bwd(const void* dy, const void* y, const uint8_t* mask, const void* x, const void* w, const float* mean,
                const float* invstd, void* dx, void* dz, void* dw, void* db, float* part, float* coef, int M, int C,
                int nrb, int relu, int dt, int dtw, int acc, hipStream_t s) {
  const int rpb = bn_rpb(M, C, nrb);
  const dim3 rg(bn_grid_x(C), nrb);
  const uint32_t nvec = (uint32_t)((size_t)M * C / 8);
  const unsigned g = bn_apply_grid(nvec);
  PRA_DISPATCH_FLOAT(dt, T, {
    if (relu)
      hipLaunchKernelGGL((bn_reduce_k<T, 1, true>), rg, dim3(kRedThreads), 0, s, (const T*)x, (const T*)dy,
                         (const T*)y, mask, mean, part, M, C, rpb);
    else
      hipLaunchKernelGGL((bn_reduce_k<T, 1, false>), rg, dim3(kRedThreads), 0, s, (const T*)x, (const T*)dy, nullptr,
                         nullptr, mean, part, M, C, rpb);
    hipLaunchKernelGGL(bn_fin_bwd_k, dim3((C + 63) / 64), dim3(1024), 0, s, part, w, dtw, mean, invstd, dw, db, coef,
                       nrb, M, C, acc);
    if (relu)
      hipLaunchKernelGGL((bn_bwd_apply_k<T, true>), dim3(g), dim3(kBnThreads), 0, s, (const T*)dy, (const T*)y, mask,
                         (const T*)x, coef, (T*)dx, (T*)dz, nvec, C);
    else
      hipLaunchKernelGGL((bn_bwd_apply_k<T, false>), dim3(g), dim3(kBnThreads), 0, s, (const T*)dy, nullptr, nullptr,
                         (const T*)x, coef, (T*)dx, (T*)dz, nvec, C);
  });
}

// Backward from the reductions a convolution's dgrad epilogue already produced (gemm_core.h
// kBnG): g is the ReLU-masked gradient, part [2][nrb][C] = per-tile sums of g and g * (x - mean).
// Finalize + apply only; the reduction pass over (dy, x, mask) is gone.
void pra_bn_bwd_parts(const void* g, const void* x, const void* w, const float* mean, const float* invstd, void* dx,
                      void* dw, void* db, const float* part, float* coef, int M, int C, int nrb, int dt, int dtw,
                      int acc, hipStream_t s) {
  const uint32_t nvec = (uint32_t)((size_t)M * C / 8);
  const unsigned gr = bn_apply_grid(nvec);
  hipLaunchKernelGGL(bn_fin_bwd_k, dim3((C + 63) / 64), dim3(1024), 0, s, part, w, dtw, mean, invstd, dw, db, coef,
                     nrb, M, C, acc);
  PRA_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL((bn_bwd_apply_k<T, false>), dim3(gr), dim3(kBnThreads), 0, s, (const T*)g, nullptr, nullptr,
                       (const T*)x, coef, (T*)dx, (T*)nullptr, nvec, C);
  });
}
}
