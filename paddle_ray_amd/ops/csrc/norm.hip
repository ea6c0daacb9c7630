// LayerNorm / RMSNorm forward+backward for gfx950.
// One workgroup per row (fwd), 16-byte vector loads, the row held in registers
// (C chunks of 8 elements per lane) so HBM is read exactly once per pass.
// Backward: grid-stride over rows with per-workgroup fp32 dW/dB partials kept in
// registers, reduced by `colsum` (deterministic, no float atomics).
#include "common.h"

namespace pra {

template <typename T, typename W, int C, bool HAS_MEAN>
__global__ void __launch_bounds__(256) norm_fwd_vec(const T* __restrict__ x, const W* __restrict__ w,
                                                    const W* __restrict__ b, T* __restrict__ y,
                                                    float* __restrict__ mean, float* __restrict__ rstd,
                                                    int cols, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const T* xr = x + (size_t)row * cols;
  T* yr = y + (size_t)row * cols;
  float v[C][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int idx = (c * nt + tid) * 8;
    if (idx < cols) {
      load8<T>(xr + idx, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
    }
  }
  float mu = 0.f;
  if (HAS_MEAN) mu = block_sum(s, red) / cols;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int idx = (c * nt + tid) * 8;
    if (idx < cols) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { float d = v[c][i] - mu; ss += d * d; }
    }
  }
  const float rs = rsqrtf(block_sum(ss, red) / cols + eps);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int idx = (c * nt + tid) * 8;
    if (idx < cols) {
      float wv[8], bv[8], o[8];
      if (w) load8<W>(w + idx, wv); else {
#pragma unroll
        for (int i = 0; i < 8; ++i) wv[i] = 1.f;
      }
      if (HAS_MEAN && b) load8<W>(b + idx, bv); else {
#pragma unroll
        for (int i = 0; i < 8; ++i) bv[i] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mu) * rs * wv[i] + bv[i];
      store8<T>(yr + idx, o);
    }
  }
  if (tid == 0) {
    if (HAS_MEAN) mean[row] = mu;
    rstd[row] = rs;
  }
}

// Scalar fallback for cols % 8 != 0 (two passes over global, L2-resident row).
template <typename T, typename W, bool HAS_MEAN>
__global__ void __launch_bounds__(256) norm_fwd_scalar(const T* __restrict__ x, const W* __restrict__ w,
                                                       const W* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ mean, float* __restrict__ rstd,
                                                       int cols, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const T* xr = x + (size_t)row * cols;
  T* yr = y + (size_t)row * cols;
  float s = 0.f;
  if (HAS_MEAN) for (int i = tid; i < cols; i += nt) s += Cvt<T>::to(xr[i]);
  float mu = HAS_MEAN ? block_sum(s, red) / cols : 0.f;
  float ss = 0.f;
  for (int i = tid; i < cols; i += nt) { float d = Cvt<T>::to(xr[i]) - mu; ss += d * d; }
  const float rs = rsqrtf(block_sum(ss, red) / cols + eps);
  for (int i = tid; i < cols; i += nt) {
    float o = (Cvt<T>::to(xr[i]) - mu) * rs;
    if (w) o *= Cvt<W>::to(w[i]);
    if (HAS_MEAN && b) o += Cvt<W>::to(b[i]);
    yr[i] = Cvt<T>::from(o);
  }
  if (tid == 0) { if (HAS_MEAN) mean[row] = mu; rstd[row] = rs; }
}

template <typename T, typename W, int C, bool HAS_MEAN>
__global__ void __launch_bounds__(256) norm_bwd_vec(const T* __restrict__ dy, const T* __restrict__ x,
                                                    const W* __restrict__ w, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, T* __restrict__ dx,
                                                    float* __restrict__ pw, float* __restrict__ pb,
                                                    int rows, int cols) {
  __shared__ float red[16];
  const int tid = threadIdx.x, nt = blockDim.x;
  float aw[C][8], ab[C][8], wv[C][8];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int idx = (c * nt + tid) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) { aw[c][i] = 0.f; ab[c][i] = 0.f; wv[c][i] = 1.f; }
    if (idx < cols && w) load8<W>(w + idx, wv[c]);
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const T* xr = x + (size_t)row * cols;
    const T* dyr = dy + (size_t)row * cols;
    const float mu = HAS_MEAN ? mean[row] : 0.f, rs = rstd[row];
    float xh[C][8], g[C][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int idx = (c * nt + tid) * 8;
      if (idx < cols) {
        float xv[8], dv[8];
        load8<T>(xr + idx, xv);
        load8<T>(dyr + idx, dv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[c][i] = (xv[i] - mu) * rs;
          g[c][i] = dv[i] * wv[c][i];
          s1 += g[c][i] * xh[c][i];
          s2 += g[c][i];
          aw[c][i] += dv[i] * xh[c][i];
          ab[c][i] += dv[i];
        }
      }
    }
    const float c1 = block_sum(s1, red) / cols;
    const float c2 = HAS_MEAN ? block_sum(s2, red) / cols : 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int idx = (c * nt + tid) * 8;
      if (idx < cols) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (g[c][i] - c2 - xh[c][i] * c1) * rs;
        store8<T>(dx + (size_t)row * cols + idx, o);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int idx = (c * nt + tid) * 8;
    if (idx < cols) {
      store8<float>(pw + (size_t)blockIdx.x * cols + idx, aw[c]);
      if (HAS_MEAN) store8<float>(pb + (size_t)blockIdx.x * cols + idx, ab[c]);
    }
  }
}

template <typename T, typename W, bool HAS_MEAN>
__global__ void __launch_bounds__(256) norm_bwd_scalar(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const W* __restrict__ w, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, T* __restrict__ dx,
                                                       float* __restrict__ pw, float* __restrict__ pb,
                                                       int rows, int cols) {
  __shared__ float red[16];
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < cols; i += nt) {
    pw[(size_t)blockIdx.x * cols + i] = 0.f;
    if (HAS_MEAN) pb[(size_t)blockIdx.x * cols + i] = 0.f;
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const T* xr = x + (size_t)row * cols;
    const T* dyr = dy + (size_t)row * cols;
    const float mu = HAS_MEAN ? mean[row] : 0.f, rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
    for (int i = tid; i < cols; i += nt) {
      float xh = (Cvt<T>::to(xr[i]) - mu) * rs, d = Cvt<T>::to(dyr[i]);
      float g = d * (w ? Cvt<W>::to(w[i]) : 1.f);
      s1 += g * xh; s2 += g;
      pw[(size_t)blockIdx.x * cols + i] += d * xh;
      if (HAS_MEAN) pb[(size_t)blockIdx.x * cols + i] += d;
    }
    const float c1 = block_sum(s1, red) / cols;
    const float c2 = HAS_MEAN ? block_sum(s2, red) / cols : 0.f;
    for (int i = tid; i < cols; i += nt) {
      float xh = (Cvt<T>::to(xr[i]) - mu) * rs, d = Cvt<T>::to(dyr[i]);
      float g = d * (w ? Cvt<W>::to(w[i]) : 1.f);
      dx[(size_t)row * cols + i] = Cvt<T>::from((g - c2 - xh * c1) * rs);
    }
  }
}

template <typename O>
__global__ void colsum_kernel(const float* __restrict__ part, O* __restrict__ out, int nblk, int cols) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[(size_t)b * cols + c];
  out[c] = Cvt<O>::from(s);
}

static int pick_threads(int cols) {
  int t = (cols / 8 + 63) / 64 * 64;
  if (t < 64) t = 64;
  if (t > 256) t = 256;
  return t;
}

template <typename T, typename W, bool HAS_MEAN>
static void launch_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                       int rows, int cols, float eps, hipStream_t s) {
  if (rows == 0) return;
  if (cols % 8 == 0) {
    int nt = pick_threads(cols);
    int chunks = (cols / 8 + nt - 1) / nt;
#define PRA_LNF(CC)                                                                                       \
  hipLaunchKernelGGL((norm_fwd_vec<T, W, CC, HAS_MEAN>), dim3(rows), dim3(nt), 0, s, (const T*)x,         \
                     (const W*)w, (const W*)b, (T*)y, mean, rstd, cols, eps)
    if (chunks <= 1) PRA_LNF(1);
    else if (chunks <= 2) PRA_LNF(2);
    else if (chunks <= 4) PRA_LNF(4);
    else if (chunks <= 8) PRA_LNF(8);
    else goto scalar;
#undef PRA_LNF
    return;
  }
scalar:
  hipLaunchKernelGGL((norm_fwd_scalar<T, W, HAS_MEAN>), dim3(rows), dim3(256), 0, s, (const T*)x,
                     (const W*)w, (const W*)b, (T*)y, mean, rstd, cols, eps);
}

template <typename T, typename W, bool HAS_MEAN>
static void launch_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                       void* dx, float* pw, float* pb, int rows, int cols, int nblk, hipStream_t s) {
  if (rows == 0) return;
  if (cols % 8 == 0) {
    int nt = pick_threads(cols);
    int chunks = (cols / 8 + nt - 1) / nt;
#define PRA_LNB(CC)                                                                                       \
  hipLaunchKernelGGL((norm_bwd_vec<T, W, CC, HAS_MEAN>), dim3(nblk), dim3(nt), 0, s, (const T*)dy,        \
                     (const T*)x, (const W*)w, mean, rstd, (T*)dx, pw, pb, rows, cols)
    if (chunks <= 1) PRA_LNB(1);
    else if (chunks <= 2) PRA_LNB(2);
    else if (chunks <= 4) PRA_LNB(4);
    else goto scalar;
#undef PRA_LNB
    return;
  }
scalar:
  hipLaunchKernelGGL((norm_bwd_scalar<T, W, HAS_MEAN>), dim3(nblk), dim3(256), 0, s, (const T*)dy,
                     (const T*)x, (const W*)w, mean, rstd, (T*)dx, pw, pb, rows, cols);
}

}  // namespace pra

using namespace pra;

#define PRA_DISPATCH_TW(dtx, dtw, ...)                                                     \
  PRA_DISPATCH_FLOAT(dtx, TX, {                                                            \
    if (dtw == dtx) { using TW = TX; __VA_ARGS__; }                                        \
    else if (dtw == kF32) { using TW = float; __VA_ARGS__; }                               \
  })

extern "C" {
void pra_layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                       int rows, int cols, float eps, int dtx, int dtw, hipStream_t s) {
  PRA_DISPATCH_TW(dtx, dtw, (launch_fwd<TX, TW, true>(x, w, b, y, mean, rstd, rows, cols, eps, s)));
}
void pra_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                       void* dx, float* pw, float* pb, int rows, int cols, int nblk, int dtx, int dtw,
                       hipStream_t s) {
  PRA_DISPATCH_TW(dtx, dtw, (launch_bwd<TX, TW, true>(dy, x, w, mean, rstd, dx, pw, pb, rows, cols, nblk, s)));
}
void pra_rmsnorm_fwd(const void* x, const void* w, void* y, float* rstd, int rows, int cols, float eps,
                     int dtx, int dtw, hipStream_t s) {
  PRA_DISPATCH_TW(dtx, dtw, (launch_fwd<TX, TW, false>(x, w, nullptr, y, nullptr, rstd, rows, cols, eps, s)));
}
void pra_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, void* dx, float* pw,
                     int rows, int cols, int nblk, int dtx, int dtw, hipStream_t s) {
  PRA_DISPATCH_TW(dtx, dtw, (launch_bwd<TX, TW, false>(dy, x, w, nullptr, rstd, dx, pw, nullptr, rows, cols, nblk, s)));
}
void pra_colsum(const float* part, void* out, int nblk, int cols, int dto, hipStream_t s) {
  PRA_DISPATCH_FLOAT(dto, TO, hipLaunchKernelGGL((colsum_kernel<TO>), dim3((cols + 255) / 256), dim3(256), 0, s,
                                                 part, (TO*)out, nblk, cols));
}
}
