// Elementwise / optimizer kernels for gfx950:
//   bias+GELU fwd/bwd (tanh or erf form), multi-tensor AdamW (one launch for a
//   whole parameter list, fp32 master weights + low-precision param write-back),
//   multi-tensor Momentum, sum-of-squares (global-norm clipping), attention
//   backward preprocess delta = rowsum(dO * O).
#include "common.h"

namespace pra {

// tanh(u) = 1 - 2 / (exp(2u) + 1): one v_exp + one v_rcp instead of libm tanhf's ~30 VALU
// (the bias-GELU backward over [tokens, 4h] was VALU-bound on tanhf); saturates to +-1 cleanly
__device__ __forceinline__ float tanh_fast(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * u) + 1.f);
}
__device__ __forceinline__ float gelu_f(float x, int approx) {
  if (approx) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    float t = tanh_fast(k0 * (x + k1 * x * x * x));
    return 0.5f * x * (1.f + t);
  }
  return gelu_erf_fast(x);
}
__device__ __forceinline__ float gelu_df(float x, int approx) {
  if (approx) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    float t = tanh_fast(k0 * (x + k1 * x * x * x));
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
  }
  return dgelu_erf_fast(x);
}

template <typename T>
__global__ void bias_gelu_fwd_k(const T* __restrict__ x, const T* __restrict__ b, T* __restrict__ y, size_t n,
                                int cols, int approx) {
  const size_t nv = n / 8;
  for (size_t v = blockIdx.x * (size_t)blockDim.x + threadIdx.x; v < nv; v += (size_t)gridDim.x * blockDim.x) {
    float a[8], bb[8];
    load8<T>(x + v * 8, a);
    if (b) load8<T>(b + (v * 8) % cols, bb);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = gelu_f(a[i] + (b ? bb[i] : 0.f), approx);
    store8<T>(y + v * 8, a);
  }
}

template <typename T>
__global__ void bias_gelu_bwd_k(const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ b,
                                T* __restrict__ dx, size_t n, int cols, int approx) {
  const size_t nv = n / 8;
  for (size_t v = blockIdx.x * (size_t)blockDim.x + threadIdx.x; v < nv; v += (size_t)gridDim.x * blockDim.x) {
    float a[8], g[8], bb[8];
    load8<T>(x + v * 8, a);
    load8<T>(dy + v * 8, g);
    if (b) load8<T>(b + (v * 8) % cols, bb);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = g[i] * gelu_df(a[i] + (b ? bb[i] : 0.f), approx);
    store8<T>(dx + v * 8, a);
  }
}

// Backward with the bias gradient fused in: grid = (column tiles of 256 x 8 columns, nrb
// row blocks); each lane owns 8 columns, walks its row block (2 rows in flight), writes dx and
// keeps the column sums of dx (= d bias) in registers -> part[nrb, cols] fp32, reduced by
// `colsum`. Removes the separate [rows, cols] re-read of dx for db.
template <typename T>
__global__ void __launch_bounds__(256) bias_gelu_bwd_db_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ b, T* __restrict__ dx,
                                                          float* __restrict__ part, int rows, int cols, int rpb,
                                                          int approx) {
  const int cv = blockIdx.x * 256 + threadIdx.x;
  if (cv * 8 >= cols) return;
  const int c = cv * 8;
  float bb[8], db[8];
  if (b) load8<T>(b + c, bb);
#pragma unroll
  for (int i = 0; i < 8; ++i) { db[i] = 0.f; if (!b) bb[i] = 0.f; }
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  int r = r0;
  // four rows (8 independent 16-B loads) in flight per lane
  for (; r + 3 < r1; r += 4) {
    float a[4][8], g[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t o = (size_t)(r + u) * cols + c;
      load8<T>(x + o, a[u]);
      load8<T>(dy + o, g[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[u][i] = g[u][i] * gelu_df(a[u][i] + bb[i], approx);
      store8<T>(dx + (size_t)(r + u) * cols + c, a[u]);
      // d bias from the ROUNDED dx values (what a separate colsum(dx) would read)
#pragma unroll
      for (int i = 0; i < 8; ++i) db[i] += Cvt<T>::to(Cvt<T>::from(a[u][i]));
    }
  }
  for (; r + 1 < r1; r += 2) {
    float a0[8], g0[8], a1[8], g1[8];
    const size_t o0 = (size_t)r * cols + c, o1 = o0 + cols;
    load8<T>(x + o0, a0);
    load8<T>(dy + o0, g0);
    load8<T>(x + o1, a1);
    load8<T>(dy + o1, g1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a0[i] = g0[i] * gelu_df(a0[i] + bb[i], approx);
      a1[i] = g1[i] * gelu_df(a1[i] + bb[i], approx);
    }
    store8<T>(dx + o0, a0);
    store8<T>(dx + o1, a1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      db[i] += Cvt<T>::to(Cvt<T>::from(a0[i])) + Cvt<T>::to(Cvt<T>::from(a1[i]));
  }
  if (r < r1) {
    float a0[8], g0[8];
    const size_t o0 = (size_t)r * cols + c;
    load8<T>(x + o0, a0);
    load8<T>(dy + o0, g0);
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = g0[i] * gelu_df(a0[i] + bb[i], approx);
    store8<T>(dx + o0, a0);
#pragma unroll
    for (int i = 0; i < 8; ++i) db[i] += Cvt<T>::to(Cvt<T>::from(a0[i]));
  }
  float* p = part + (size_t)blockIdx.y * cols + c;
  *reinterpret_cast<float4*>(p) = make_float4(db[0], db[1], db[2], db[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(db[4], db[5], db[6], db[7]);
}

// Column partial sums of a [rows, cols] matrix (a Linear's bias gradient = colsum(dy)):
// grid = (column tiles of 256 x 8 columns, nrb row blocks); each lane owns 8 columns and keeps
// four 16-B row loads in flight -> part[nrb, cols] fp32, reduced by colsum16 (which can add the
// result straight into an existing .grad). Replaces a generic reduce at ~4 TB/s.
template <typename T>
__global__ void __launch_bounds__(256) colsum_rows_k(const T* __restrict__ x, float* __restrict__ part, int rows,
                                                     int cols, int rpb) {
  const int cv = blockIdx.x * 256 + threadIdx.x;
  if (cv * 8 >= cols) return;
  const int c = cv * 8;
  float s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = 0.f;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  int r = r0;
  for (; r + 3 < r1; r += 4) {
    float a[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load8<T>(x + (size_t)(r + u) * cols + c, a[u]);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] += (a[0][i] + a[1][i]) + (a[2][i] + a[3][i]);
  }
  for (; r < r1; ++r) {
    float a[8];
    load8<T>(x + (size_t)r * cols + c, a);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] += a[i];
  }
  float* p = part + (size_t)blockIdx.y * cols + c;
  *reinterpret_cast<float4*>(p) = make_float4(s[0], s[1], s[2], s[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(s[4], s[5], s[6], s[7]);
}

template <typename T>
__global__ void bias_gelu_fwd_scalar(const T* __restrict__ x, const T* __restrict__ b, T* __restrict__ y, size_t n,
                                     int cols, int approx) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = Cvt<T>::from(gelu_f(Cvt<T>::to(x[i]) + (b ? Cvt<T>::to(b[i % cols]) : 0.f), approx));
}
template <typename T>
__global__ void bias_gelu_bwd_scalar(const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ b,
                                     T* __restrict__ dx, size_t n, int cols, int approx) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dx[i] = Cvt<T>::from(Cvt<T>::to(dy[i]) *
                         gelu_df(Cvt<T>::to(x[i]) + (b ? Cvt<T>::to(b[i % cols]) : 0.f), approx));
}

// ---------------------------------------------------------------------------
// multi-tensor AdamW
// tab[t] = {master_or_param, grad, m, v, lowp_param (0 if none), n, grad_dtype, param_dtype}
// ftab[t] = {weight_decay, lr_mul, -, -};  chunks[c] = {tensor, start}
// ---------------------------------------------------------------------------
constexpr int kChunk = 65536;

__device__ __forceinline__ float ld_any(const void* p, size_t i, int dt) {
  if (dt == kF32) return ((const float*)p)[i];
  if (dt == kBF16) return bf2f(((const uint16_t*)p)[i]);
  return (float)((const f16*)p)[i];
}
__device__ __forceinline__ void st_any(void* p, size_t i, int dt, float v) {
  if (dt == kF32) ((float*)p)[i] = v;
  else if (dt == kBF16) ((uint16_t*)p)[i] = f2bf(v);
  else ((f16*)p)[i] = (f16)v;
}

// Vector body of the common mixed-precision case (bf16 or fp32 grad, fp32 master, optional
// bf16 low-precision param copy): 4 elements per lane per step, 16-B fp32 accesses.
template <bool BF16G, bool LOWP>
__device__ __forceinline__ void adamw_vec4(float* __restrict__ master, const void* __restrict__ grad,
                                           float* __restrict__ m, float* __restrict__ v, uint16_t* __restrict__ lowp,
                                           int64_t start, int64_t end, float b1, float b2, float eps, float decay,
                                           float step, float rbc2, float gscale) {
  for (int64_t i = start + 4 * threadIdx.x; i + 3 < end; i += 4 * blockDim.x) {
    float g[4];
    if (BF16G) {
      const uint2 u = *reinterpret_cast<const uint2*>((const uint16_t*)grad + i);
      g[0] = __uint_as_float(u.x << 16); g[1] = __uint_as_float(u.x & 0xffff0000u);
      g[2] = __uint_as_float(u.y << 16); g[3] = __uint_as_float(u.y & 0xffff0000u);
    } else {
      const float4 u = *reinterpret_cast<const float4*>((const float*)grad + i);
      g[0] = u.x; g[1] = u.y; g[2] = u.z; g[3] = u.w;
    }
    float4 mv = *reinterpret_cast<float4*>(m + i);
    float4 vv = *reinterpret_cast<float4*>(v + i);
    float4 pv = *reinterpret_cast<float4*>(master + i);
    float mm[4] = {mv.x, mv.y, mv.z, mv.w}, vq[4] = {vv.x, vv.y, vv.z, vv.w}, pp[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = g[k] * gscale;
      mm[k] = b1 * mm[k] + (1.f - b1) * gk;
      vq[k] = b2 * vq[k] + (1.f - b2) * gk * gk;
      pp[k] = pp[k] * decay - step * mm[k] / (sqrtf(vq[k] * rbc2) + eps);
    }
    *reinterpret_cast<float4*>(m + i) = make_float4(mm[0], mm[1], mm[2], mm[3]);
    *reinterpret_cast<float4*>(v + i) = make_float4(vq[0], vq[1], vq[2], vq[3]);
    *reinterpret_cast<float4*>(master + i) = make_float4(pp[0], pp[1], pp[2], pp[3]);
    if (LOWP) *reinterpret_cast<uint2*>(lowp + i) = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
  }
}

// gscale_ptr (device, nullable): global-norm clip coefficient read in-kernel, so the clip
// needs no separate pass over the gradients.
__global__ void __launch_bounds__(256) adamw_mt_k(const int64_t* __restrict__ tab, const float* __restrict__ ftab,
                                                  const int64_t* __restrict__ chunks, float lr, float b1, float b2,
                                                  float eps, float bc1, float bc2, float gscale,
                                                  const float* __restrict__ gscale_ptr) {
  if (gscale_ptr) gscale *= *gscale_ptr;
  const int64_t t = chunks[2 * blockIdx.x];
  int64_t start = chunks[2 * blockIdx.x + 1];
  const int64_t* d = tab + 8 * t;
  void* master = (void*)d[0];
  const void* grad = (const void*)d[1];
  float* m = (float*)d[2];
  float* v = (float*)d[3];
  void* lowp = (void*)d[4];
  const int64_t n = d[5];
  const int gdt = (int)d[6], pdt = (int)d[7];
  const int mdt = lowp ? kF32 : pdt;
  const float wd = ftab[4 * t], lrt = lr * ftab[4 * t + 1];
  const float decay = 1.f - lrt * wd, step = lrt / bc1, rbc2 = 1.f / bc2;
  int64_t end = start + kChunk;
  if (end > n) end = n;
  const bool aligned = ((start & 3) == 0) && ((((uintptr_t)master | (uintptr_t)m | (uintptr_t)v) & 15) == 0) &&
                       ((((uintptr_t)grad | (uintptr_t)lowp) & 7) == 0);
  if (aligned && mdt == kF32 && (gdt == kBF16 || gdt == kF32) && (!lowp || pdt == kBF16)) {
    const int64_t vend = start + ((end - start) & ~(int64_t)3);
    if (gdt == kBF16) {
      if (lowp) adamw_vec4<true, true>((float*)master, grad, m, v, (uint16_t*)lowp, start, vend, b1, b2, eps,
                                       decay, step, rbc2, gscale);
      else adamw_vec4<true, false>((float*)master, grad, m, v, nullptr, start, vend, b1, b2, eps, decay, step,
                                   rbc2, gscale);
    } else {
      if (lowp) adamw_vec4<false, true>((float*)master, grad, m, v, (uint16_t*)lowp, start, vend, b1, b2, eps,
                                        decay, step, rbc2, gscale);
      else adamw_vec4<false, false>((float*)master, grad, m, v, nullptr, start, vend, b1, b2, eps, decay, step,
                                    rbc2, gscale);
    }
    start = vend;  // scalar tail below
  }
  for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) {
    float g = ld_any(grad, i, gdt) * gscale;
    float mi = b1 * m[i] + (1.f - b1) * g;
    float vi = b2 * v[i] + (1.f - b2) * g * g;
    m[i] = mi;
    v[i] = vi;
    float p = ld_any(master, i, mdt) * decay - step * mi / (sqrtf(vi * rbc2) + eps);
    st_any(master, i, mdt, p);
    if (lowp) st_any(lowp, i, pdt, p);
  }
}

// Multi-tensor zero fill (optimizer.clear_grad): one launch for every gradient instead of one
// fill kernel per tensor (ResNet-50: ~180 tiny launches per step). ch[2b] = address of block b's
// piece, ch[2b + 1] = its byte count (<= 64 KB); 16-B stores where aligned, bytes for the tail.
__global__ void __launch_bounds__(256) zero_mt_k(const int64_t* __restrict__ ch) {
  char* p = reinterpret_cast<char*>(ch[2 * blockIdx.x]);
  const int64_t n = ch[2 * blockIdx.x + 1];
  const int64_t n16 = (reinterpret_cast<uintptr_t>(p) & 15) == 0 ? n / 16 : 0;
  for (int64_t i = threadIdx.x; i < n16; i += blockDim.x) reinterpret_cast<uint4*>(p)[i] = make_uint4(0, 0, 0, 0);
  for (int64_t i = n16 * 16 + threadIdx.x; i < n; i += blockDim.x) p[i] = 0;
}

// tab[t] = {master_or_param, grad, velocity, 0, lowp, n, gdt, pdt}; ftab = {wd, lr_mul}
__global__ void __launch_bounds__(256) momentum_mt_k(const int64_t* __restrict__ tab, const float* __restrict__ ftab,
                                                     const int64_t* __restrict__ chunks, float lr, float mu,
                                                     int nesterov, float gscale,
                                                     const float* __restrict__ gscale_ptr) {
  if (gscale_ptr) gscale *= *gscale_ptr;
  const int64_t t = chunks[2 * blockIdx.x], start = chunks[2 * blockIdx.x + 1];
  const int64_t* d = tab + 8 * t;
  void* master = (void*)d[0];
  const void* grad = (const void*)d[1];
  float* vel = (float*)d[2];
  void* lowp = (void*)d[4];
  const int64_t n = d[5];
  const int gdt = (int)d[6], pdt = (int)d[7];
  const int mdt = lowp ? kF32 : pdt;
  const float wd = ftab[4 * t], lrt = lr * ftab[4 * t + 1];
  int64_t end = start + kChunk;
  if (end > n) end = n;
  for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) {
    float p = ld_any(master, i, mdt);
    float g = ld_any(grad, i, gdt) * gscale + wd * p;
    float vi = mu * vel[i] + g;
    vel[i] = vi;
    p -= lrt * (nesterov ? g + mu * vi : vi);
    st_any(master, i, mdt, p);
    if (lowp) st_any(lowp, i, pdt, p);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) sumsq_vec_k(const T* __restrict__ x, float* __restrict__ out, size_t n) {
  __shared__ float red[16];
  float s = 0.f;
  const size_t nv = n / 8;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  // eight independent 16-B loads in flight per lane (one at a time left HBM half idle); the
  // grid is capped at one workgroup per CU so the closing same-address atomics stay few
  // (thousands of them serialise at the memory-side atomic unit)
  for (; i + 7 * stride < nv; i += 8 * stride) {
    float v[8][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) load8<T>(x + (i + u * stride) * 8, v[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[u][j] * v[u][j];
  }
  for (; i < nv; i += stride) {
    float v[8];
    load8<T>(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  if (blockIdx.x == 0)
    for (size_t i = nv * 8 + threadIdx.x; i < n; i += blockDim.x) { float v = Cvt<T>::to(x[i]); s += v * v; }
  s = block_sum(s, red);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

template <typename T>
__global__ void __launch_bounds__(256) sumsq_k(const T* __restrict__ x, float* __restrict__ out, size_t n) {
  __shared__ float red[16];
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float v = Cvt<T>::to(x[i]);
    s += v * v;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

// delta[b,h,s] = sum_d dO[b,s,h,d] * O[b,s,h,d]   (O, dO contiguous [B,S,H,D]).
// D/8 lanes per row with 16-B loads (D=128: 16 lanes, 4 rows per wave).
template <typename T>
__global__ void __launch_bounds__(256) attn_delta_k(const T* __restrict__ o, const T* __restrict__ dO,
                                                    float* __restrict__ delta, int B, int H, int S, int D) {
  const int lpr = D / 8;  // lanes per row (power of two, <= 64)
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / lpr;
  const int sub = threadIdx.x % lpr;
  const bool valid = r < (int64_t)B * S * H;
  float s = 0.f;
  if (valid) {
    float a[8], g[8];
    load8<T>(o + r * D + sub * 8, a);
    load8<T>(dO + r * D + sub * 8, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] * g[i];
  }
  for (int off = lpr / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (valid && sub == 0) {  // rows < 2^31 (host-checked): 32-bit index math, not 64-bit emulated division
    const int ri = (int)r, h = ri % H, bs = ri / H, sq = bs % S, b = bs / S;
    delta[((int64_t)b * H + h) * S + sq] = s;
  }
}

static int grid_for(size_t nv) {
  size_t g = (nv + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace pra

using namespace pra;

extern "C" {
void pra_bias_gelu_fwd(const void* x, const void* b, void* y, int64_t rows, int cols, int dt, int approx,
                       hipStream_t s) {
  size_t n = (size_t)rows * cols;
  if (!n) return;
  if (cols % 8 == 0) {
    PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((bias_gelu_fwd_k<T>), dim3(grid_for(n / 8)), dim3(256), 0, s,
                                                 (const T*)x, (const T*)b, (T*)y, n, cols, approx));
  } else {
    PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((bias_gelu_fwd_scalar<T>), dim3(grid_for(n)), dim3(256), 0, s,
                                                 (const T*)x, (const T*)b, (T*)y, n, cols, approx));
  }
}
void pra_bias_gelu_bwd(const void* dy, const void* x, const void* b, void* dx, int64_t rows, int cols, int dt,
                       int approx, hipStream_t s) {
  size_t n = (size_t)rows * cols;
  if (!n) return;
  if (cols % 8 == 0) {
    PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((bias_gelu_bwd_k<T>), dim3(grid_for(n / 8)), dim3(256), 0, s,
                                                 (const T*)dy, (const T*)x, (const T*)b, (T*)dx, n, cols, approx));
  } else {
    PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((bias_gelu_bwd_scalar<T>), dim3(grid_for(n)), dim3(256), 0, s,
                                                 (const T*)dy, (const T*)x, (const T*)b, (T*)dx, n, cols, approx));
  }
}
void pra_adamw_mt(const int64_t* tab, const float* ftab, const int64_t* chunks, int nchunks, float lr, float b1,
                  float b2, float eps, float bc1, float bc2, float gscale, const float* gscale_ptr, hipStream_t s) {
  if (!nchunks) return;
  hipLaunchKernelGGL(adamw_mt_k, dim3(nchunks), dim3(256), 0, s, tab, ftab, chunks, lr, b1, b2, eps, bc1, bc2,
                     gscale, gscale_ptr);
}
void pra_zero_mt(const int64_t* chunks, int nchunks, hipStream_t s) {
  if (nchunks > 0) hipLaunchKernelGGL(zero_mt_k, dim3(nchunks), dim3(256), 0, s, chunks);
}
void pra_momentum_mt(const int64_t* tab, const float* ftab, const int64_t* chunks, int nchunks, float lr, float mu,
                     int nesterov, float gscale, const float* gscale_ptr, hipStream_t s) {
  if (!nchunks) return;
  hipLaunchKernelGGL(momentum_mt_k, dim3(nchunks), dim3(256), 0, s, tab, ftab, chunks, lr, mu, nesterov, gscale,
                     gscale_ptr);
}
void pra_sumsq_accum(const void* x, float* out, int64_t n, int dt, hipStream_t s) {
  if (!n) return;
  if (((uintptr_t)x & 15) == 0) {
    int g = grid_for((size_t)n / 8);
    if (g > 256) g = 256;
    PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((sumsq_vec_k<T>), dim3(g), dim3(256), 0, s, (const T*)x, out,
                                                 (size_t)n));
  } else {
    PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((sumsq_k<T>), dim3(grid_for(n) > 1024 ? 1024 : grid_for(n)),
                                                 dim3(256), 0, s, (const T*)x, out, (size_t)n));
  }
}
void pra_flash_bwd_pre(const void* o, const void* dO, float* delta, int B, int H, int S, int D, int dt,
                       hipStream_t s) {
  int64_t rows = (int64_t)B * S * H;
  if (!rows || rows >= (1ll << 31)) return;
  const int64_t threads = rows * (D / 8);
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((attn_delta_k<T>), dim3((threads + 255) / 256), dim3(256), 0, s,
                                               (const T*)o, (const T*)dO, delta, B, H, S, D));
}
void pra_bias_gelu_bwd_db(const void* dy, const void* x, const void* b, void* dx, float* part, int rows, int cols,
                          int nrb, int dt, int approx, hipStream_t s) {
  if (!rows || cols % 8) return;
  const int rpb = (rows + nrb - 1) / nrb;
  const dim3 grid((cols / 8 + 255) / 256, nrb);
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((bias_gelu_bwd_db_k<T>), grid, dim3(256), 0, s, (const T*)dy,
                                               (const T*)x, (const T*)b, (T*)dx, part, rows, cols, rpb, approx));
}
void pra_colsum_rows(const void* x, float* part, int rows, int cols, int nrb, int dt, hipStream_t s) {
  if (!rows || cols % 8) return;
  const int rpb = (rows + nrb - 1) / nrb;
  const dim3 grid((cols / 8 + 255) / 256, nrb);
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((colsum_rows_k<T>), grid, dim3(256), 0, s, (const T*)x, part, rows,
                                               cols, rpb));
}
}
