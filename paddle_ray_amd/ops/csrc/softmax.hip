// Row softmax fwd/bwd and fused softmax + cross-entropy fwd/bwd for gfx950.
// One workgroup per row; online (max, sum) in a single streaming pass with
// 16-byte loads; CE backward writes dlogits = (softmax - onehot) * dloss in one
// pass (the [tokens, vocab] probability matrix is never materialised).
#include "common.h"

namespace pra {

__device__ __forceinline__ void ms_combine(float& m, float& s, float m2, float s2) {
  float M = fmaxf(m, m2);
  float a = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  float b = (m2 == -INFINITY) ? 0.f : s2 * __expf(m2 - M);
  m = M;
  s = a + b;
}

__device__ __forceinline__ void block_ms(float& m, float& s, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    ms_combine(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) { red[2 * wid] = m; red[2 * wid + 1] = s; }
  __syncthreads();
  m = -INFINITY; s = 0.f;
  for (int i = 0; i < nw; ++i) ms_combine(m, s, red[2 * i], red[2 * i + 1]);
}

template <typename T>
__device__ __forceinline__ void row_ms(const T* xr, int cols, float& m, float& s) {
  const int tid = threadIdx.x, nt = blockDim.x;
  m = -INFINITY; s = 0.f;
  if ((cols & 7) == 0) {
    for (int idx = tid * 8; idx < cols; idx += nt * 8) {
      float v[8];
      load8<T>(xr + idx, v);
      float lm = v[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) lm = fmaxf(lm, v[i]);
      float ls = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) ls += __expf(v[i] - lm);
      ms_combine(m, s, lm, ls);
    }
  } else {
    for (int i = tid; i < cols; i += nt) ms_combine(m, s, Cvt<T>::to(xr[i]), 1.f);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) softmax_fwd_k(const T* __restrict__ x, T* __restrict__ y, int cols) {
  __shared__ float red[32];
  const size_t row = blockIdx.x;
  const T* xr = x + row * cols;
  T* yr = y + row * cols;
  float m, s;
  row_ms<T>(xr, cols, m, s);
  block_ms(m, s, red);
  const float inv = 1.f / s;
  const int tid = threadIdx.x, nt = blockDim.x;
  if ((cols & 7) == 0) {
    for (int idx = tid * 8; idx < cols; idx += nt * 8) {
      float v[8];
      load8<T>(xr + idx, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = __expf(v[i] - m) * inv;
      store8<T>(yr + idx, v);
    }
  } else {
    for (int i = tid; i < cols; i += nt) yr[i] = Cvt<T>::from(__expf(Cvt<T>::to(xr[i]) - m) * inv);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) softmax_bwd_k(const T* __restrict__ y, const T* __restrict__ dy,
                                                     T* __restrict__ dx, int cols) {
  __shared__ float red[16];
  const size_t row = blockIdx.x;
  const T* yr = y + row * cols;
  const T* dyr = dy + row * cols;
  T* dxr = dx + row * cols;
  const int tid = threadIdx.x, nt = blockDim.x;
  float dot = 0.f;
  if ((cols & 7) == 0) {
    for (int idx = tid * 8; idx < cols; idx += nt * 8) {
      float a[8], b[8];
      load8<T>(yr + idx, a);
      load8<T>(dyr + idx, b);
#pragma unroll
      for (int i = 0; i < 8; ++i) dot += a[i] * b[i];
    }
  } else {
    for (int i = tid; i < cols; i += nt) dot += Cvt<T>::to(yr[i]) * Cvt<T>::to(dyr[i]);
  }
  dot = block_sum(dot, red);
  if ((cols & 7) == 0) {
    for (int idx = tid * 8; idx < cols; idx += nt * 8) {
      float a[8], b[8];
      load8<T>(yr + idx, a);
      load8<T>(dyr + idx, b);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = a[i] * (b[i] - dot);
      store8<T>(dxr + idx, a);
    }
  } else {
    for (int i = tid; i < cols; i += nt)
      dxr[i] = Cvt<T>::from(Cvt<T>::to(yr[i]) * (Cvt<T>::to(dyr[i]) - dot));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) ce_fwd_k(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                int ignore_index) {
  __shared__ float red[32];
  const size_t row = blockIdx.x;
  const T* xr = logits + row * V;
  float m, s;
  row_ms<T>(xr, V, m, s);
  block_ms(m, s, red);
  if (threadIdx.x == 0) {
    const float lse = m + __logf(s);
    lse_out[row] = lse;
    const int64_t lab = labels[row];
    if (lab == ignore_index || lab < 0 || lab >= V) loss[row] = 0.f;
    else loss[row] = lse - Cvt<T>::to(xr[lab]);
  }
}

// Vocab-parallel CE, pass 1: this rank's slice [start, start + V) of each row gives its
// partial (max, sum exp(x - max), picked logit) — 3 floats/row, all-gathered over the TP
// group (a [world, rows, 3] tensor) instead of reducing [rows, V] probabilities.
template <typename T>
__global__ void __launch_bounds__(256) ce_part_fwd_k(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                     float* __restrict__ stats, int V, int64_t start) {
  __shared__ float red[32];
  const size_t row = blockIdx.x;
  const T* xr = logits + row * V;
  float m, s;
  row_ms<T>(xr, V, m, s);
  block_ms(m, s, red);
  if (threadIdx.x == 0) {
    const int64_t lab = labels[row] - start;
    stats[row * 3 + 0] = m;
    stats[row * 3 + 1] = s;
    stats[row * 3 + 2] = (lab >= 0 && lab < V) ? Cvt<T>::to(xr[lab]) : 0.f;
  }
}

// pass 2: combine the world's partials per row -> loss, lse (one thread per row).
__global__ void __launch_bounds__(256) ce_part_final_k(const float* __restrict__ stats, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss, float* __restrict__ lse_out, int rows,
                                                       int world, int64_t vtot, int ignore_index) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float m = -INFINITY, s = 0.f, picked = 0.f;
  for (int r = 0; r < world; ++r) {
    const float* st = stats + ((size_t)r * rows + row) * 3;
    ms_combine(m, s, st[0], st[1]);
    picked += st[2];
  }
  const float lse = m + __logf(s);
  lse_out[row] = lse;
  const int64_t lab = labels[row];
  loss[row] = (lab == ignore_index || lab < 0 || lab >= vtot) ? 0.f : lse - picked;
}

// dlogits = (exp(x - lse) - onehot(label - start)) * dloss for this rank's V columns
// (start = 0, vtot = V for the unsharded op). dl may alias logits (each element is read and
// written by the same lane).
template <typename T>
__global__ void __launch_bounds__(256) ce_bwd_k(const T* logits, const int64_t* __restrict__ labels,
                                                const float* __restrict__ lse, const float* __restrict__ dloss,
                                                T* dl, int V, int ignore_index, int gx, int64_t start, int64_t vtot) {
  const size_t row = blockIdx.x / gx;
  const int part = blockIdx.x % gx;
  const T* xr = logits + row * V;
  T* gr = dl + row * V;
  const int64_t glab = labels[row];
  const bool valid = !(glab == ignore_index || glab < 0 || glab >= vtot);
  const int64_t lab = glab - start;
  const float g = valid ? dloss[row] : 0.f;
  const float L = lse[row];
  const int stride = gx * blockDim.x * 8;
  if ((V & 7) == 0) {
    for (int idx = (part * blockDim.x + threadIdx.x) * 8; idx < V; idx += stride) {
      float v[8];
      load8<T>(xr + idx, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float p = __expf(v[i] - L);
        if (idx + i == lab) p -= 1.f;
        v[i] = p * g;
      }
      store8<T>(gr + idx, v);
    }
  } else {
    for (int i = part * blockDim.x + threadIdx.x; i < V; i += gx * blockDim.x) {
      float p = __expf(Cvt<T>::to(xr[i]) - L);
      if (i == lab) p -= 1.f;
      gr[i] = Cvt<T>::from(p * g);
    }
  }
}

static int nthreads_for(int cols) {
  int t = (cols / 8 + 63) / 64 * 64;
  return t < 64 ? 64 : (t > 256 ? 256 : t);
}

}  // namespace pra

using namespace pra;

extern "C" {
void pra_softmax_fwd(const void* x, void* y, int rows, int cols, int dt, hipStream_t s) {
  if (!rows) return;
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((softmax_fwd_k<T>), dim3(rows), dim3(nthreads_for(cols)), 0, s,
                                               (const T*)x, (T*)y, cols));
}
void pra_softmax_bwd(const void* y, const void* dy, void* dx, int rows, int cols, int dt, hipStream_t s) {
  if (!rows) return;
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((softmax_bwd_k<T>), dim3(rows), dim3(nthreads_for(cols)), 0, s,
                                               (const T*)y, (const T*)dy, (T*)dx, cols));
}
void pra_softmax_ce_fwd(const void* logits, const int64_t* labels, float* loss, float* lse, int rows, int V,
                        int ignore_index, int dt, hipStream_t s) {
  if (!rows) return;
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((ce_fwd_k<T>), dim3(rows), dim3(256), 0, s, (const T*)logits,
                                               labels, loss, lse, V, ignore_index));
}
void pra_softmax_ce_bwd(const void* logits, const int64_t* labels, const float* lse, const float* dloss, void* dl,
                        int rows, int V, int ignore_index, int dt, hipStream_t s) {
  if (!rows) return;
  int gx = (V / 8 + 255) / 256;
  if (gx > 8) gx = 8;
  if (gx < 1) gx = 1;
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((ce_bwd_k<T>), dim3(gx * rows), dim3(256), 0, s, (const T*)logits,
                                               labels, lse, dloss, (T*)dl, V, ignore_index, gx, (int64_t)0,
                                               (int64_t)V));
}
void pra_vp_ce_part_fwd(const void* logits, const int64_t* labels, float* stats, int rows, int V, int64_t start,
                        int dt, hipStream_t s) {
  if (!rows) return;
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((ce_part_fwd_k<T>), dim3(rows), dim3(256), 0, s, (const T*)logits,
                                               labels, stats, V, start));
}
void pra_vp_ce_final(const float* stats, const int64_t* labels, float* loss, float* lse, int rows, int world,
                     int64_t vtot, int ignore_index, hipStream_t s) {
  if (!rows) return;
  hipLaunchKernelGGL(ce_part_final_k, dim3((rows + 255) / 256), dim3(256), 0, s, stats, labels, loss, lse, rows,
                     world, vtot, ignore_index);
}
void pra_vp_ce_bwd(const void* logits, const int64_t* labels, const float* lse, const float* dloss, void* dl,
                   int rows, int V, int64_t start, int64_t vtot, int ignore_index, int dt, hipStream_t s) {
  if (!rows) return;
  int gx = (V / 8 + 255) / 256;
  if (gx > 8) gx = 8;
  if (gx < 1) gx = 1;
  PRA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((ce_bwd_k<T>), dim3(gx * rows), dim3(256), 0, s, (const T*)logits,
                                               labels, lse, dloss, (T*)dl, V, ignore_index, gx, start, vtot));
}
}
